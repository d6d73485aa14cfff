// context.hpp -- libpgrt's host-side frame state, shared by the translation units of the C ABI
// (internal: not installed, not part of include/pgrt.h).
//   context.cpp      the C ABI core: contexts, configuration, scene / camera, synchronous and
//                    asynchronous renders, batch ray queries, the frame sink
//   scene.cpp        set_scene (host packing, on-device BVH build) and the camera
//   frame.cpp        frame scheduling: pipeline slots, the tile deal, the per-level launch
//                    sequence (enqueue_frame), counters, overflow re-render, frame statistics
//   distributed.cpp  multi-GPU: the gather over RCCL, the overflow agreement, the single-process
//                    multi-device context, the distributed C ABI
//   diagnostics.cpp  launch timeline, per-level diagnostics, math self-tests
//   tiles_abi.cpp    the host-only tile deal / unpack C ABI (no HIP: sanitizer builds)
// Replaces SimpleGuiDX11::Producer's serial y/x loop over Raytracer::get_pixel
// (APP/simpleguidx11.cpp:95-125, APP/raytracer.cpp:396-437) with wavefront passes on HIP streams,
// and Embree's scene API (APP/raytracer.cpp:71-127) with an on-device BVH.  No exception crosses
// the ABI: every entry point returns a PGRT_* code and records a message readable with
// pgrt_last_error().
#pragma once

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "trace.hpp"
#include "camera_ops.hpp"
#include "shade_ray.hpp"
#include "path.hpp"
#include "tiles.hpp"
#include "stamps.hpp"

namespace pgrt {

// level-0 rays per sample batch (pgrt_config default): r3ag A/B 16M / 32M / 64M: C3 10.53 / 10.26 /
// 10.12 ms, C4 40.6 / 38.4 / 38.8 ms (fewer batches: each pays its deep-level chain once)
constexpr long long kMaxBatchRays = 32ll << 20;
constexpr int kTraceGridThreads = 2048 * 256;    // persistent trace grid (global overflow stacks)
constexpr int kMaxFramesInFlight = 16;
constexpr long long kStampWaves = 4ll << 20;  // timeline: wave stamps per frame set (64 MB)
constexpr int kMaxFramesPerCall = 64;

struct StageTimer {
    struct Rec {
        hipEvent_t a, b;
        int cat, cat2;  // cat2: optional second bucket (per-level time), -1 none
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    bool on = false;
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        PGRT_HIP(hipEventCreate(&e));
        return e;
    }
    int begin(hipStream_t s, int cat, int cat2 = -1) {
        if (!on) return -1;
        Rec r{get(), get(), cat, cat2};
        PGRT_HIP(hipEventRecord(r.a, s));
        recs.push_back(r);
        return (int)recs.size() - 1;
    }
    void end(hipStream_t s, int id) {
        if (id >= 0) PGRT_HIP(hipEventRecord(recs[id].b, s));
    }
    // a closest-hit launch: its kernel records the pair itself (set_trace_events); nothing
    // launched -> both recorded here (zero time)
    int begin_kernel(int cat, int cat2 = -1) {
        if (!on) return -1;
        recs.push_back(Rec{get(), get(), cat, cat2});
        const int id = (int)recs.size() - 1;
        set_trace_events(recs[id].a, recs[id].b);
        return id;
    }
    void end_kernel(hipStream_t s, int id, bool launched) {
        set_trace_events(nullptr, nullptr);
        if (id >= 0 && !launched) {
            PGRT_HIP(hipEventRecord(recs[id].a, s));
            PGRT_HIP(hipEventRecord(recs[id].b, s));
        }
    }
    void collect(double* ms) {  // after stream sync
        for (auto& r : recs) {
            float t = 0;
            PGRT_HIP(hipEventElapsedTime(&t, r.a, r.b));
            ms[r.cat] += t;
            if (r.cat2 >= 0) ms[r.cat2] += t;
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        recs.clear();
    }
    ~StageTimer() {
        for (auto& r : recs) {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

enum { CAT_RAYGEN, CAT_TRACE, CAT_SHADE, CAT_SHADOW, CAT_COMBINE, CAT_LTRACE, CAT_LSHADE = CAT_LTRACE + kMaxLevels,
       CAT_N = CAT_LSHADE + kMaxLevels };

// One pipeline instance: queues, level nodes, shadow queue and counters for a subset of the
// frame's tiles, enqueued on its own stream.  Two slots run concurrently: each launch of one
// slot fills the CUs the other slot's latency-bound launches leave idle (the tail of every
// level, the deep Whitted levels).  r1 A/B on C2: 1 slot 0.87 ms, 2 slots 0.79-0.80, 3 slots
// 0.80, 4+ slots slower (more streams than the 4 hardware queues); a stagger (slot k+1 waits for
// slot k's level 0) was slower (0.90).
struct FrameSlot {
    hipStream_t stream = nullptr;
    hipEvent_t ev_done = nullptr;
    DevBuf<int4> tiles;
    DevBuf<float4> q_ro[2], q_rd[2], q_hit[2];
    DevBuf<float> q_time[2];
    DevBuf<int> q_defer;          // rays a budgeted packet launch handed to the 8-lane kernel
    DevBuf<float4> probe_hits;    // the AUTO probe's side launch: its hit records and deferrals (discarded)
    DevBuf<int> probe_defer;
    DevBuf<unsigned long long> l0_hit, l0_pending;  // 1-spp level-0 wave masks (L0Final)
    int q_cap = 0;
    std::vector<std::unique_ptr<DevBuf<float4>>> n_color, n_att;
    std::vector<std::unique_ptr<DevBuf<int4>>> n_link;
    std::vector<int> level_cap;
    DevBuf<float4> s_ro, s_rd, s_hit, s_contrib;
    DevBuf<unsigned char> s_lit;
    int s_cap = 0;
    DevBuf<FrameCounters> fc;  // one per sample batch
    std::vector<FrameCounters> host_fc;
    // pinned staging (async copies from pageable memory would block the enqueue of the next slot)
    FrameCounters* pinned_fc = nullptr;
    int pinned_fc_n = 0;
    int4* pinned_tiles = nullptr;
    int pinned_tiles_n = 0;
    // per-tile deep flags of a synchronous frame (FrameParams::tile_deep), zeroed by the export
    DevBuf<int> tile_deep;
    int* pinned_deep = nullptr;
    int pinned_deep_n = 0;
    void ensure_pinned(int batches, int ntiles) {
        if (pinned_fc_n < batches) {
            if (pinned_fc) (void)hipHostFree(pinned_fc);
            // written by the export kernel (coherent: no host-side cache maintenance)
            PGRT_HIP(hipHostMalloc((void**)&pinned_fc, sizeof(FrameCounters) * batches,
                                   hipHostMallocMapped | hipHostMallocCoherent));
            pinned_fc_n = batches;
        }
        if (pinned_tiles_n < ntiles) {
            if (pinned_tiles) (void)hipHostFree(pinned_tiles);
            PGRT_HIP(hipHostMalloc((void**)&pinned_tiles, sizeof(int4) * ntiles, hipHostMallocDefault));
            pinned_tiles_n = ntiles;
        }
    }
    // the deep flags of ntiles tiles: device copy zeroed once (the export kernel re-zeroes it)
    void ensure_deep(int ntiles, hipStream_t s) {
        if (pinned_deep_n < ntiles) {
            if (pinned_deep) (void)hipHostFree(pinned_deep);
            PGRT_HIP(hipHostMalloc((void**)&pinned_deep, sizeof(int) * ntiles,
                                   hipHostMallocMapped | hipHostMallocCoherent));
            pinned_deep_n = ntiles;
        }
        if (tile_deep.n < (size_t)ntiles) {
            tile_deep.alloc(ntiles);
            PGRT_HIP(hipMemsetAsync(tile_deep.p, 0, sizeof(int) * tile_deep.n, s));
        }
    }
    DevBuf<float4> accum;
    DevBuf<int> gstack;
    std::vector<int4> tiles_dev;  // host copy of the device tile list
    int expect_count[kMaxLevels] = {0};  // grid hints from the previous frame (0 = unknown)
    int expect_defer[kMaxLevels] = {0};
    int expect_shadow_total = 0;
    int sub_first = -1;  // the last frame's subtree level (its shadow rays never enter the shadow queue)
    // first: the frame's slot 0 -- the deep tiles of a synchronous frame (deal_tiles), whose chain
    // of small latency-bound launches is the frame's critical path -- on a high-priority stream,
    // so its launches take CUs before slot 1's level-0 blocks
    explicit FrameSlot(bool first) {
        int lo = 0, hi = 0;
        PGRT_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        PGRT_HIP(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, first ? hi : lo));
        PGRT_HIP(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
    }
    ~FrameSlot() {
        if (pinned_fc) (void)hipHostFree(pinned_fc);
        if (pinned_tiles) (void)hipHostFree(pinned_tiles);
        if (pinned_deep) (void)hipHostFree(pinned_deep);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// One frame in flight: its pipeline slots, the frame's arguments (kept for an overflow re-render)
// and, for a distributed frame, this rank's tile-compact buffer.  Frames in flight run
// concurrently on their own slot streams: the deep Whitted levels of one frame are chains of
// dependent launches over a few thousand rays (latency floors), and the next
// frame's wide levels fill the CUs they leave idle.
struct FrameSet {
    std::vector<std::unique_ptr<FrameSlot>> slots;
    // recorded on the context stream after the last reader of this set's output (gather/unpack):
    // the set's next frame waits for it before overwriting its buffers
    hipEvent_t ev_ready = nullptr;
    bool pending = false, has_result = false;
    unsigned long long ticket = 0;
    pgrt_render_params params{};
    std::vector<int4> tiles;
    float* out = nullptr;
    int out_mode = 0, ox = 0, oy = 0, pitch = 0;
    int K = 0;             // slots of the pending frame
    int batches = 0;       // sample batches the pending frame enqueued (all slots)
    int nframes = 1;       // consecutive frames rendered by this call (tiles repeated per frame)
    int frame_tiles = 0;   // tiles of one frame in `tiles` (nframes > 1)
    int frame_out_tiles = 0;  // tiles per frame in the tile-compact output (>= frame_tiles)
    long long frame_stride = 0;  // floats between frames of a framebuffer output
    bool distributed = false;
    TileDeal deal{1, 1, 1};  // distributed: the tile deal this frame was rendered with
    float* dist_fb = nullptr;
    DevBuf<float> tilebuf;  // distributed: this rank's tiles, tile-compact
    // host-output frames (pgrt_render, pgrt_render_frames_host_async; set_host_output): rendered
    // into a device framebuffer (host_src: host_stage, or the context's out_tmp), then moved to
    // host_dst.  A page-locked destination (host_map: its device-visible address) is written by one
    // export kernel per pipeline slot as soon as that slot's tiles are final (k_export_tiles), so
    // the bulk slot's pixels cross PCIe while the deep-tile slot still renders; a pageable one gets
    // ONE device-to-host copy of host_bytes after every slot, on slot 0's stream
    DevBuf<float> host_stage;
    float* host_src = nullptr;
    float* host_dst = nullptr;
    float* host_map = nullptr;
    size_t host_bytes = 0;
    // PGRT_HOST_EXPORT_SPLIT: the blit kernel's share runs on host_aux beside slot 0's DMA copy
    hipStream_t host_aux = nullptr;
    hipEvent_t ev_host0 = nullptr, ev_host1 = nullptr;
    int cam_w = 0, cam_h = 0;  // image size at submission (the gather's layout)
    bool deep_rec = false;     // the level-0 shades record deep tiles (FrameParams::tile_deep)
    pgrt_stats stats{};
    std::chrono::steady_clock::time_point t0;
    // distributed frames: device time of the gather (ncclGather, including the wait for the
    // slowest peer) and of rank 0's unpack, read when the frame is waited for
    hipEvent_t ev_g0 = nullptr, ev_g1 = nullptr, ev_g2 = nullptr;
    bool gather_timed = false;
    // multi-process distributed frames, rank 0: every peer's overflow flag (the tail of its send,
    // copied to host memory behind the unpack, ev_flags) -- the re-render agreement without a
    // control collective
    hipEvent_t ev_flags = nullptr;
    int* peer_flags = nullptr;  // pinned: kMaxRanks flag words, then kMaxRanks sequence words
    unsigned gather_seq = 0;    // this rank's distributed-frame sequence number of the frame
    bool poison = false;        // this rank gave up on the frame (its send carries flag 2)
    // a re-gather after an overflow (rank 0): receive / unpack only the ranks marked here
    bool regather = false;
    char regather_peer[kMaxRanks] = {};
    // launch timeline (pgrt_timeline_enable): this call's wave stamps and the launches they belong to
    DevBuf<unsigned long long> stamps;
    std::vector<StampLaunch> stamp_launches;
    long long stamp_used = 0;
    bool stamp_overflow = false;  // the call had more waves than the buffer: later launches unrecorded
    FrameSet() {
        PGRT_HIP(hipEventCreateWithFlags(&ev_ready, hipEventDisableTiming));
        PGRT_HIP(hipEventCreate(&ev_g0));
        PGRT_HIP(hipEventCreate(&ev_g1));
        PGRT_HIP(hipEventCreate(&ev_g2));
        PGRT_HIP(hipEventCreateWithFlags(&ev_flags, hipEventDisableTiming));
        PGRT_HIP(hipHostMalloc((void**)&peer_flags, sizeof(int) * 2 * kMaxRanks, hipHostMallocMapped | hipHostMallocCoherent));
        std::fill(peer_flags, peer_flags + 2 * kMaxRanks, 0);
    }
    ~FrameSet() {
        for (auto& s : slots)
            if (s->stream) (void)hipStreamSynchronize(s->stream);
        if (host_aux) (void)hipStreamSynchronize(host_aux);
        for (hipEvent_t e : {ev_ready, ev_g0, ev_g1, ev_g2, ev_flags, ev_host0, ev_host1})
            if (e) (void)hipEventDestroy(e);
        if (host_aux) (void)hipStreamDestroy(host_aux);
        if (peer_flags) (void)hipHostFree(peer_flags);
    }
};
}  // namespace pgrt

using namespace pgrt;  // internal header: the ABI's opaque context is built from pgrt's types

struct pgrt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // scene
    DevBuf<float4> tri;
    DevBuf<BvhNode> nodes;
    DevBuf<Bvh8Node> nodes8;
    DevBuf<float4> tri8;  // triangles in 8-wide leaf order
    DevBuf<float4> tri_ng;  // Ng per binary-order reference (packet traversal)
    DevBuf<float> attr;
    DevBuf<unsigned char> prim_glass;
    DevBuf<DevMaterial> mats;
    DevBuf<DevTexture> texd;
    DevBuf<unsigned char> texels;
    DevBuf<DevLight> lights;
    SceneView view{};
    float light0[3] = {0, 0, 0};  // the first light's position (compact shadow queues)
    bool has_scene = false;
    pgrt_config cfg{};  // pgrt_set_config (zero = defaults)
    // PGRT_PACKETS_AUTO: bit L = level L traced as wave packets.  Level 0 always (8x8 pixel
    // blocks are coherent by construction); deeper levels by their measured packet utilisation
    // (the fraction of the wave's node stream a lane's ray needed, FrameCounters::pkt): on while
    // it stays >= kPacketMinUtil, re-probed every kPacketProbeFrames frames while off.  Start:
    // levels 0-2 (k_shade queues each wave's reflections and refractions as separate
    // pixel-ordered groups; r1g C2: packets on levels 0 / 0-1 / 0-2 / 0-3 / all: 0.206 / 0.197 /
    // 0.194 / 0.196 / 0.202 ms/frame)
    unsigned auto_packets = 0x7u;
    double packet_util[kMaxLevels] = {};  // last measured utilisation per level (0 = never measured)
    unsigned long long frames_collected = 0;
    int probe_level = -1;  // level traced as packets in the next frame to refresh its utilisation
    // pgrt_config.tile_order: the image tiles (64x64 grid of a deep_w x deep_h frame) whose
    // primary rays hit a dielectric in the last synchronous frame of that size
    std::vector<unsigned char> deep_tiles;
    int deep_w = 0, deep_h = 0;
    pgrt_bvh_info info{};

    CameraView cam{};
    bool has_cam = false;

    // frame state: frames in flight (set 0 serves the synchronous entry points), each with its
    // independent pipeline slots (tile subsets) on their own streams
    std::vector<std::unique_ptr<FrameSet>> sets;
    // pgrt_config.call_order: recorded after a call's level-0 shade; the next call's level-0
    // trace waits for it (calls in flight take the GPU's bulk work in submission order)
    hipEvent_t l0_token = nullptr;
    bool l0_token_live = false;
    int frames_in_flight = 1;
    unsigned long long next_ticket = 1;
    DevBuf<int> gstack;        // pgrt_intersect_closest
    DevBuf<float> out_tmp;
    StageTimer timer;
    bool timeline_on = false;                     // pgrt_timeline_enable
    std::vector<pgrt_timeline_rec> timeline;      // collected launch records (pgrt_timeline_read)
    std::vector<unsigned long long> stamp_host;   // staging of a frame set's stamps
    std::vector<FrameCounters> last_fc;  // per slot and batch, for pgrt_frame_diag
    double level_ms[kMaxLevels][2] = {};  // per-level trace / shade ms of the last profiled call

    // multi-GPU
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0;
    unsigned gather_count = 0;  // distributed frames submitted (the gather tail's sequence number)
    // non-empty once rank 0's bounded wait for the peers' tiles ran out: the communicator was
    // aborted (ncclCommAbort ends the pending ncclRecv, so the context stream drains), the frames
    // in flight were dropped, and every later distributed call fails at once with this reason
    std::string comm_aborted;
    // PGRT_EMULATE_RANK=r/N (measurement tool only, no communicator): distributed frames render
    // rank r's share of an N-GPU frame on this device; the gather becomes a device copy of this
    // rank's tiles into a full-size gather buffer (+ the unpack on rank 0), so one GPU measures a
    // rank's compute and rank 0's unpack at N GPUs without the xGMI transfer
    bool emulated = false;
    DevBuf<float> tilebuf, gathered, fb_dev;
    // single-process multi-device context (pgrt_create_devices): this context is
    // rank 0 and owns one member context per further device (rank r = members[r - 1]); every
    // frame renders each rank's tiles on its device and gathers them here.  Communicators from
    // ncclCommInitAll over distinct devices; ranks that share a device (peer_copy) exchange
    // their tiles by device copies instead (RCCL takes one rank per device)
    bool group = false;
    bool peer_copy = false;
    std::vector<pgrt_ctx*> members;

    // frame sink (progressive accumulation)
    DevBuf<float> acc_frame, acc_sum, acc_mean;
    int acc_count = 0, acc_w = 0, acc_h = 0;

    ~pgrt_ctx() {
        if (group && comm) {
            // communicators of one ncclCommInitAll: finalised together in one group (each
            // finalize may wait on its peers), then destroyed one by one
            for (pgrt_ctx* m : members) {
                (void)hipSetDevice(m->device);
                if (m->stream) (void)hipStreamSynchronize(m->stream);
            }
            (void)hipSetDevice(device);
            if (stream) (void)hipStreamSynchronize(stream);
            (void)ncclGroupStart();
            (void)ncclCommFinalize(comm);
            for (pgrt_ctx* m : members)
                if (m->comm) (void)ncclCommFinalize(m->comm);
            (void)ncclGroupEnd();
        }
        for (pgrt_ctx* m : members) {
            (void)hipSetDevice(m->device);
            if (m->stream) (void)hipStreamSynchronize(m->stream);
            delete m;
        }
        (void)hipSetDevice(device);
        if (l0_token) (void)hipEventDestroy(l0_token);
        if (comm) (void)ncclCommDestroy(comm);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace pgrt {

template <class F>
int guarded(pgrt_ctx* ctx, F&& f) {
    try {
        if (ctx) {
            PGRT_HIP(hipSetDevice(ctx->device));
        }
        f();
        return PGRT_OK;
    } catch (const Error& e) {
        if (ctx) ctx->err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        if (ctx) ctx->err = "host out of memory";
        return PGRT_ERR_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        if (ctx) ctx->err = e.what();
        return PGRT_ERR_INVALID_ARGUMENT;
    }
}

// ---- scene.cpp
CameraView make_camera(const pgrt_camera& c);
void set_scene(pgrt_ctx* ctx, const pgrt_scene_desc* d);

// ---- frame.cpp
FrameSet* frame_set(pgrt_ctx* ctx, int i);
long long batch_rays(const pgrt_ctx* ctx);
int group_max(const pgrt_ctx* ctx);
void enqueue_frame(pgrt_ctx* ctx, FrameSet* fs);
bool read_frame_counters(pgrt_ctx* ctx, FrameSet* fs);
void rerender_frame(pgrt_ctx* ctx, FrameSet* fs, bool grow, int& retries);
void frame_stats(pgrt_ctx* ctx, FrameSet* fs, int retries);
void finish_frame(pgrt_ctx* ctx, FrameSet* fs);
void finish_through(pgrt_ctx* ctx, unsigned long long last);
void drain_frames(pgrt_ctx* ctx);
void start_frame(pgrt_ctx* ctx, FrameSet* fs, const pgrt_render_params* p, std::vector<int4> tiles, float* out,
                 int out_mode, int ox, int oy, int pitch, bool distributed, float* fb, int nframes = 1,
                 long long frame_stride = 0, TileDeal deal = TileDeal{1, 1, 1}, bool defer_gather = false);
void render_tiles(pgrt_ctx* ctx, const pgrt_render_params* p, const std::vector<int4>& tiles, float* out,
                  int out_mode, int ox, int oy, int pitch, pgrt_stats* st, int nframes = 1,
                  long long frame_stride = 0, float* host_out = nullptr, size_t host_bytes = 0);
std::vector<int4> rect_tiles(int x0, int y0, int w, int h);
void set_host_output(FrameSet* fs, float* dst, float* src, size_t bytes);
void frame_rect(const pgrt_ctx* ctx, const pgrt_render_params* p, int& x, int& y, int& w, int& h);

// ---- distributed.cpp
void collect_frame(pgrt_ctx* ctx, FrameSet* fs);
void check_comm(const pgrt_ctx* ctx);
void gather_frame(pgrt_ctx* ctx, FrameSet* fs);
void gather_times(FrameSet* fs, pgrt_stats* st);
TileDeal ctx_deal(const pgrt_ctx* ctx, int world);
std::vector<int4> rank_tiles(int W, int H, int rank, const TileDeal& d);
void on_device(const pgrt_ctx* c);
std::vector<pgrt_ctx*> group_ranks(pgrt_ctx* head);
void group_finish_through(pgrt_ctx* head, unsigned long long last);
unsigned long long group_submit(pgrt_ctx* head, const pgrt_render_params* p, int nframes, float* fb);
void group_render(pgrt_ctx* head, const pgrt_render_params* p, int nframes, float* fb, pgrt_stats* st);

// ---- diagnostics.cpp
void collect_timeline(pgrt_ctx* ctx, FrameSet* fs);

}  // namespace pgrt
