// context.cpp -- frame driver and C ABI (include/pgrt.h) of libpgrt.
//
// Replaces SimpleGuiDX11::Producer's serial y/x loop over Raytracer::get_pixel
// (APP/simpleguidx11.cpp:95-125, APP/raytracer.cpp:396-437) with one wavefront pass per
// sample batch on one HIP stream, and Embree's scene API (APP/raytracer.cpp:71-127) with an
// on-device LBVH.  No exception crosses the ABI: every entry point returns a PGRT_* code and
// records a message readable with pgrt_last_error().
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

using namespace pgrt;

namespace pgrt {
namespace {
thread_local StampLog* t_stamp_log = nullptr;
}
void set_stamp_log(StampLog* log) { t_stamp_log = log; }
StampLog* stamp_log() { return t_stamp_log; }
}  // namespace pgrt

namespace {

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

}  // namespace

namespace pgrt {

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
    // host-output frames (pgrt_render_frames_host_async): rendered into host_stage, then ONE
    // device-to-host copy of host_bytes into host_dst on the set's first slot stream, overlapped
    // with the frames in flight behind it
    DevBuf<float> host_stage;
    float* host_dst = nullptr;
    size_t host_bytes = 0;
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
    int* peer_flags = nullptr;  // pinned, kMaxRanks words
    // a re-gather after an overflow (rank 0): receive / unpack only the ranks marked here
    bool regather = false;
    char regather_peer[kMaxRanks] = {};
    // launch timeline (pgrt_timeline_enable): this call's wave stamps and the launches they belong to
    DevBuf<unsigned long long> stamps;
    std::vector<StampLaunch> stamp_launches;
    long long stamp_used = 0;
    FrameSet() {
        PGRT_HIP(hipEventCreateWithFlags(&ev_ready, hipEventDisableTiming));
        PGRT_HIP(hipEventCreate(&ev_g0));
        PGRT_HIP(hipEventCreate(&ev_g1));
        PGRT_HIP(hipEventCreate(&ev_g2));
        PGRT_HIP(hipEventCreateWithFlags(&ev_flags, hipEventDisableTiming));
        PGRT_HIP(hipHostMalloc((void**)&peer_flags, sizeof(int) * kMaxRanks, hipHostMallocMapped | hipHostMallocCoherent));
        std::fill(peer_flags, peer_flags + kMaxRanks, 0);
    }
    ~FrameSet() {
        for (auto& s : slots)
            if (s->stream) (void)hipStreamSynchronize(s->stream);
        for (hipEvent_t e : {ev_ready, ev_g0, ev_g1, ev_g2, ev_flags})
            if (e) (void)hipEventDestroy(e);
        if (peer_flags) (void)hipHostFree(peer_flags);
    }
};
}  // namespace pgrt

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

namespace {

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

// PinHoleCamera::PinHoleCamera (APP/PinHoleCamera.cpp:5-29), evaluated on the host in float.
CameraView make_camera(const pgrt_camera& c) {
    auto norm = [](float v[3]) {
        const float n = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        if (n != 0) {
            const float rn = 1 / std::sqrt(n);
            v[0] *= rn;
            v[1] *= rn;
            v[2] *= rn;
        }
    };
    auto cross = [](const float a[3], const float b[3], float o[3]) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    CameraView k{};
    k.width = c.width;
    k.height = c.height;
    k.fy = (float)c.height / (2 * tanf(c.fov_y / 2));
    for (int i = 0; i < 3; ++i) k.from[i] = c.from[i];
    float z[3] = {c.from[0] - c.at[0], c.from[1] - c.at[1], c.from[2] - c.at[2]};
    float x[3], y[3];
    cross(c.up, z, x);
    cross(z, x, y);
    norm(z);
    norm(x);
    norm(y);
    k.m[0] = x[0]; k.m[1] = y[0]; k.m[2] = z[0];
    k.m[3] = x[1]; k.m[4] = y[1]; k.m[5] = z[1];
    k.m[6] = x[2]; k.m[7] = y[2]; k.m[8] = z[2];
    return k;
}

void set_scene(pgrt_ctx* ctx, const pgrt_scene_desc* d) {
    PGRT_REQUIRE(d != nullptr, PGRT_ERR_INVALID_ARGUMENT, "scene descriptor is NULL");
    // An empty scene (an OBJ without faces: Embree commits it and every rtcIntersect1 misses, so
    // every pixel is the environment, raytracer.cpp:390-393) becomes one zero-area placeholder
    // triangle at the origin: Ng = 0, so the closest-hit test never accepts it, and every layout
    // and kernel path stays the non-empty one.  pgrt_bvh_info reports 0 triangles.
    static const float kZero9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, kZero6[6] = {0, 0, 0, 0, 0, 0};
    static const int kMat0 = 0;
    static const pgrt_material kDefaultMat = {{0.4f, 0.4f, 0.4f}, {0.8f, 0.8f, 0.8f}, 1.0f, 1.5f, 0, -1};
    pgrt_scene_desc placeholder;
    const bool empty = d->num_triangles == 0;
    if (empty) {
        placeholder = *d;
        placeholder.num_triangles = 1;
        placeholder.positions = kZero9;
        placeholder.normals = kZero9;
        placeholder.uvs = kZero6;
        placeholder.material_ids = &kMat0;
        if (placeholder.num_materials == 0) {
            placeholder.num_materials = 1;
            placeholder.materials = &kDefaultMat;
        }
        d = &placeholder;
    }
    const int n = d->num_triangles;
    PGRT_REQUIRE(n > 0 && n < (1 << 27), PGRT_ERR_INVALID_ARGUMENT, "num_triangles must be in [0, 2^27)");
    PGRT_REQUIRE(d->positions && d->normals && d->uvs && d->material_ids, PGRT_ERR_INVALID_ARGUMENT,
                 "triangle arrays must be non-NULL");
    PGRT_REQUIRE(d->num_materials > 0 && d->materials, PGRT_ERR_INVALID_ARGUMENT, "at least one material required");
    PGRT_REQUIRE(d->num_lights >= 0 && d->num_lights <= 64 && (d->num_lights == 0 || d->lights),
                 PGRT_ERR_INVALID_ARGUMENT, "num_lights must be in [0, 64]");
    PGRT_REQUIRE(d->num_textures >= 0 && (d->num_textures == 0 || d->textures), PGRT_ERR_INVALID_ARGUMENT,
                 "bad texture table");
    PGRT_REQUIRE(d->env_texture < d->num_textures, PGRT_ERR_INVALID_ARGUMENT, "env_texture out of range");
    auto t0 = std::chrono::steady_clock::now();
    hipStream_t st = ctx->stream;
    ctx->has_scene = false;

    // materials / textures / lights (host-side packing, small)
    std::vector<DevMaterial> mats(d->num_materials);
    for (int i = 0; i < d->num_materials; ++i) {
        const pgrt_material& m = d->materials[i];
        DevMaterial& o = mats[i];
        for (int k = 0; k < 3; ++k) {
            o.kd[k] = m.diffuse[k];
            o.ks[k] = m.specular[k];
        }
        o.ns = m.shininess;
        o.ior = m.ior;
        o.type = m.type;
        o.tex = m.diffuse_tex;
        PGRT_REQUIRE(m.diffuse_tex < d->num_textures, PGRT_ERR_INVALID_ARGUMENT, "diffuse_tex out of range");
    }
    std::vector<DevTexture> texs(std::max(1, d->num_textures));
    long long pool = 0;
    for (int i = 0; i < d->num_textures; ++i) {
        const pgrt_texture& t = d->textures[i];
        PGRT_REQUIRE(t.width > 0 && t.height > 0 && t.bpp >= 3 && t.pitch >= t.width * t.bpp && t.data,
                     PGRT_ERR_INVALID_ARGUMENT, "bad texture " + std::to_string(i));
        texs[i] = DevTexture{t.width, t.height, t.pitch, t.bpp, pool, (long long)t.pitch * t.height};
        pool += ((long long)t.pitch * t.height + 255) / 256 * 256;
    }
    if (d->num_lights > 0)
        for (int k = 0; k < 3; ++k) ctx->light0[k] = d->lights[0].position[k];
    std::vector<DevLight> lights(std::max(1, d->num_lights));
    for (int i = 0; i < d->num_lights; ++i)
        for (int k = 0; k < 3; ++k) {
            lights[i].pos[k] = d->lights[i].position[k];
            lights[i].kd[k] = d->lights[i].diffuse[k];
            lights[i].ks[k] = d->lights[i].specular[k];
        }
    // per-triangle shading attributes in original order: n0 n1 n2 uv0 uv1 uv2 material
    std::vector<float> attr((size_t)n * 16);
    float lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (int i = 0; i < n; ++i) {
        float* a = &attr[(size_t)i * 16];
        std::memcpy(a, d->normals + (size_t)i * 9, 9 * sizeof(float));
        std::memcpy(a + 9, d->uvs + (size_t)i * 6, 6 * sizeof(float));
        int mid = d->material_ids[i];
        if (mid < 0 || mid >= d->num_materials) mid = 0;  // see DESIGN.md: NULL surface material
        std::memcpy(a + 15, &mid, sizeof(int));
        for (int v = 0; v < 9; ++v) {
            const float p = d->positions[(size_t)i * 9 + v];
            lo[v % 3] = std::min(lo[v % 3], p);
            hi[v % 3] = std::max(hi[v % 3], p);
        }
    }
    float ext = 0;
    for (int k = 0; k < 3; ++k) ext = std::max(ext, hi[k] - lo[k]);
    PGRT_REQUIRE(std::isfinite(ext), PGRT_ERR_INVALID_ARGUMENT, "non-finite vertex positions");
    const float pad = 1e-5f * ext + 1e-30f;

    ctx->attr.alloc(attr.size());
    PGRT_HIP(hipMemcpyAsync(ctx->attr.p, attr.data(), attr.size() * sizeof(float), hipMemcpyHostToDevice, st));
    // per-triangle "dielectric" byte: the shadow resolve's is_illuminated test reads one byte
    // instead of the attribute line + the material table (two dependent loads fewer)
    std::vector<unsigned char> glass((size_t)std::max(1, n), 0);
    for (int i = 0; i < n; ++i) {
        int mid;
        std::memcpy(&mid, &attr[(size_t)i * 16 + 15], sizeof(int));
        glass[i] = mats[mid].type == PGRT_MATERIAL_DIELECTRIC ? 1 : 0;
    }
    ctx->prim_glass.alloc(glass.size());
    PGRT_HIP(hipMemcpyAsync(ctx->prim_glass.p, glass.data(), glass.size(), hipMemcpyHostToDevice, st));
    ctx->mats.alloc(mats.size());
    PGRT_HIP(hipMemcpyAsync(ctx->mats.p, mats.data(), mats.size() * sizeof(DevMaterial), hipMemcpyHostToDevice, st));
    ctx->texd.alloc(texs.size());
    PGRT_HIP(hipMemcpyAsync(ctx->texd.p, texs.data(), texs.size() * sizeof(DevTexture), hipMemcpyHostToDevice, st));
    ctx->texels.alloc((size_t)std::max(1ll, pool) + 16);  // + the 12-byte texel window's overhang (shade_ops.hpp)
    for (int i = 0; i < d->num_textures; ++i)
        PGRT_HIP(hipMemcpyAsync(ctx->texels.p + texs[i].offset, d->textures[i].data, (size_t)texs[i].size,
                                hipMemcpyHostToDevice, st));
    ctx->lights.alloc(lights.size());
    PGRT_HIP(hipMemcpyAsync(ctx->lights.p, lights.data(), lights.size() * sizeof(DevLight), hipMemcpyHostToDevice, st));

    // positions -> device, LBVH build on device
    DevBuf<float> pos;
    pos.alloc((size_t)n * 9);
    PGRT_HIP(hipMemcpyAsync(pos.p, d->positions, (size_t)n * 9 * sizeof(float), hipMemcpyHostToDevice, st));
    BuildOut bo{};
    // layout choices (pgrt_config): builder, traversal width, split budget
    const pgrt_config& cfg = ctx->cfg;
    const int builder = cfg.bvh_builder == PGRT_BVH_LBVH || n < 2 ? kBuilderLbvh : kBuilderPloc;
    const int width = cfg.bvh_width == 8 ? 8 : 2;
    const float beta = std::max(0.0f, std::min(4.0f, cfg.split_beta));
    bo.builder = builder;
    bo.leaf_max = kLeafMaxTris;
    auto tb = std::chrono::steady_clock::now();
    if (builder == kBuilderPloc) {
        build_ploc_refs(pos.p, n, beta, pad, ext, ctx->tri, ctx->nodes, &bo, st);
    } else {
        ctx->tri.alloc((size_t)n * 3);
        ctx->nodes.alloc((size_t)std::max(1, n - 1));
        DevBuf<int> scratch;
        scratch.alloc(lbvh_scratch_ints(n));
        const size_t tmp_bytes = lbvh_sort_temp_bytes(n);
        DevBuf<unsigned char> sort_tmp;
        sort_tmp.alloc(tmp_bytes);
        build_lbvh(pos.p, n, ctx->tri.p, ctx->nodes.p, scratch.p, sort_tmp.p, tmp_bytes, pad, &bo, st);
    }
    const int m = bo.refs;
    // the 8-wide layout is always built: the multi-lane kernel traces small (deep-level) queues
    // over it; PGRT_BVH_WIDTH=8 also sends the big queues to the one-lane 8-wide kernel
    int wide_nodes = 0, wide_depth = 0;
    {
        ctx->nodes8.alloc((size_t)std::max(1, m));
        ctx->tri8.alloc((size_t)m * 3);
        const float4 rlo = make_float4(lo[0] - pad, lo[1] - pad, lo[2] - pad, 0.0f);
        const float4 rhi = make_float4(hi[0] + pad, hi[1] + pad, hi[2] + pad, 0.0f);
        build_bvh8(ctx->nodes.p, ctx->tri.p, bo.root, m, rlo, rhi, ctx->nodes8.p, ctx->tri8.p, &wide_nodes,
                   &wide_depth, st);
    }
    ctx->tri_ng.alloc((size_t)std::max(1, m));
    compute_tri_normals(ctx->tri.p, m, ctx->tri_ng.p, st);
    auto te = std::chrono::steady_clock::now();
    PGRT_REQUIRE(bo.max_depth <= kLdsStack + kGlobalStack - 2, PGRT_ERR_INVALID_ARGUMENT,
                 "BVH depth " + std::to_string(bo.max_depth) + " exceeds the traversal stack");

    SceneView& v = ctx->view;
    v.tri = ctx->tri.p;
    v.tri_ng = ctx->tri_ng.p;
    v.nodes = ctx->nodes.p;
    v.root = bo.root;
    v.nodes8 = ctx->nodes8.p;
    v.tri8 = ctx->tri8.p;
    v.depth8 = wide_depth;
    v.group_max = kDefaultGroupMax;  // per frame: pgrt_config.group_max / frames in flight
    v.wide = width == 8 ? 1 : 0;
    v.ntri = n;
    v.depth = bo.max_depth;
    v.attr = ctx->attr.p;
    v.prim_glass = ctx->prim_glass.p;
    v.mats = ctx->mats.p;
    v.tex = ctx->texd.p;
    v.nmat = (int)mats.size();
    v.ntex = (int)texs.size();
    v.texels = ctx->texels.p;
    v.env = d->env_texture;
    v.nlight = d->num_lights;
    v.lights = ctx->lights.p;
    ctx->has_scene = true;
    // AUTO's packet choice starts over for a new scene: levels 0-2 on packets, level 0 only for
    // big scenes (their bounce levels are incoherent: r2 / r3 measured AUTO turning 1-2 off
    // after a start frame of multi-ms packet launches)
    ctx->auto_packets = n > kPacketBigScene ? 0x1u : 0x7u;
    ctx->probe_level = -1;
    ctx->frames_collected = 0;
    std::fill(ctx->packet_util, ctx->packet_util + kMaxLevels, 0.0);
    pgrt_bvh_info& bi = ctx->info;
    bi.num_triangles = empty ? 0 : n;
    bi.num_nodes = width == 8 ? wide_nodes : bo.num_nodes;
    bi.max_depth = width == 8 ? wide_depth : bo.max_depth;
    bi.width = width;
    bi.build_ms = std::chrono::duration<double, std::milli>(te - tb).count();
    bi.builder = bo.builder;
    bi.build_iterations = bo.iterations;
    bi.num_references = bo.refs;
    bi.split_beta = builder == kBuilderPloc ? beta : 0.0f;
    for (int k = 0; k < 3; ++k) {
        bi.scene_lo[k] = lo[k];
        bi.scene_hi[k] = hi[k];
    }
    bi.device_bytes = ctx->tri.bytes() + ctx->tri_ng.bytes() + ctx->tri8.bytes() + ctx->nodes8.bytes() + ctx->nodes.bytes() +
                      ctx->attr.bytes() + ctx->texels.bytes();
    (void)t0;
}

void ensure_frame_buffers(FrameSlot* sl, int n0, int levels, int nlight, int batches) {
    if (sl->q_cap < n0) {
        for (int b = 0; b < 2; ++b) {
            sl->q_ro[b].alloc(n0);
            sl->q_rd[b].alloc(n0);
            sl->q_hit[b].alloc(n0);
            sl->q_time[b].alloc(n0);
        }
        sl->l0_hit.alloc((size_t)n0 / 64 + 1);
        sl->l0_pending.alloc((size_t)n0 / 64 + 1);
        sl->q_defer.alloc(n0);
        sl->q_cap = n0;
    }
    if ((int)sl->level_cap.size() < levels) sl->level_cap.resize(levels, 0);
    while ((int)sl->n_color.size() < levels) {
        sl->n_color.emplace_back(new DevBuf<float4>());
        sl->n_att.emplace_back(new DevBuf<float4>());
        sl->n_link.emplace_back(new DevBuf<int4>());
    }
    for (int L = 0; L < levels; ++L) {
        const int cap = std::max(L == 0 ? n0 : std::min(sl->q_cap, std::max(sl->level_cap[L], n0)), 1);
        if (sl->level_cap[L] < cap || (int)sl->n_color[L]->n < cap) {
            sl->n_color[L]->alloc(cap);
            sl->n_att[L]->alloc(cap);
            sl->n_link[L]->alloc(cap);
            sl->level_cap[L] = cap;
        }
    }
    const int nl = std::max(1, nlight);
    if (sl->s_cap < n0 * nl) {
        const int sc = n0 * nl;
        sl->s_ro.alloc(sc);
        sl->s_rd.alloc(sc);
        sl->s_hit.alloc(sc);
        sl->s_contrib.alloc(sc);
        sl->s_lit.alloc(sc);
        sl->s_cap = sc;
    }
    if (sl->fc.n < (size_t)batches) {  // zeroed once; every frame's export kernel re-zeroes them
        sl->fc.alloc((size_t)batches);
        // on the slot's own (non-blocking) stream, ahead of the frame's kernels: a NULL-stream
        // hipMemset is not ordered with them and could zero a running frame's queue counters
        PGRT_HIP(hipMemsetAsync(sl->fc.p, 0, sizeof(FrameCounters) * batches, sl->stream));
    }
    if (sl->gstack.n == 0) sl->gstack.alloc((size_t)kTraceGridThreads * kGlobalStack);
}

// grow a slot's level queues / shadow queue after an overflow (2x what was requested)
void grow_after_overflow(FrameSlot* sl, int levels) {
    int shadow_need = 0;
    for (auto& h : sl->host_fc) {
        int sc = 0;
        for (int L = 0; L < kMaxLevels; ++L) sc += fc_shadow(h, L);
        shadow_need = std::max(shadow_need, sc);
        for (int L = 1; L < levels; ++L) {
            const int need = fc_count(h, L) * 2;
            if (need > sl->level_cap[L]) sl->level_cap[L] = need;
            if (need > sl->q_cap) {
                for (int b = 0; b < 2; ++b) {
                    sl->q_ro[b].alloc(need);
                    sl->q_rd[b].alloc(need);
                    sl->q_hit[b].alloc(need);
                    sl->q_time[b].alloc(need);
                }
                sl->q_defer.alloc(need);
                sl->q_cap = need;
            }
        }
    }
    for (int L = 1; L < levels; ++L)
        if ((int)sl->n_color[L]->n < sl->level_cap[L]) {
            sl->n_color[L]->alloc(sl->level_cap[L]);
            sl->n_att[L]->alloc(sl->level_cap[L]);
            sl->n_link[L]->alloc(sl->level_cap[L]);
        }
    if (shadow_need * 2 > sl->s_cap) {
        const int sh = shadow_need * 2;
        sl->s_ro.alloc(sh);
        sl->s_rd.alloc(sh);
        sl->s_hit.alloc(sh);
        sl->s_contrib.alloc(sh);
        sl->s_lit.alloc(sh);
        sl->s_cap = sh;
    }
}

// PGRT_DEBUG_SYNC=1: synchronise after every launch of the frame pipeline and name the launch
// that failed (a device fault is otherwise reported by whichever HIP call comes next)
void debug_sync(hipStream_t s, const char* what, int level, int batch) {
    static const bool on = getenv("PGRT_DEBUG_SYNC") != nullptr;
    if (!on) return;
    hipError_t e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess)
        throw Error(PGRT_ERR_HIP, std::string(what) + " (level " + std::to_string(level) + ", batch " +
                                      std::to_string(batch) + "): " + hipGetErrorString(e));
}

FrameSet* frame_set(pgrt_ctx* ctx, int i) {
    while ((int)ctx->sets.size() <= i) {
        ctx->sets.emplace_back(new FrameSet());
        PGRT_HIP(hipEventRecord(ctx->sets.back()->ev_ready, ctx->stream));
    }
    return ctx->sets[i].get();
}

// level-0 rays per sample batch
long long batch_rays(const pgrt_ctx* ctx) {
    return ctx->cfg.max_batch_rays > 0 ? ctx->cfg.max_batch_rays : kMaxBatchRays;
}

// is level L traced as wave packets (pgrt_config.packet_levels)
bool packet_level(const pgrt_ctx* ctx, int L) {
    const int k = ctx->cfg.packet_levels;
    if (k == PGRT_PACKETS_OFF) return false;
    // (profiled frames never probe: their traversal counts describe the timed frames' choice)
    if (k == PGRT_PACKETS_AUTO)
        return L == 0 || ((ctx->auto_packets >> L) & 1u) != 0;
    return L < k;
}

// AUTO's probe of a level that is off packets: a SIDE packet launch over the level's first
// kProbeRays rays (hit records discarded, deferred rays not finished) samples the utilisation; the
// level itself is traced as usual, so a probe frame costs one bounded launch instead of a whole
// level on packets (C5's incoherent level 1: multi-ms resume launches, profiles/r3 verdict)
constexpr int kProbeRays = 65536;

// PGRT_PACKETS_AUTO: a level stays on wave packets while its rays use at least this fraction of
// the wave's node stream (calibrated on C2 / C5), re-probed while off
constexpr double kPacketMinUtil = 0.4;
// hysteresis: a level on packets leaves them only below this utilisation (C2's level 2 measures
// ~0.44 and would otherwise flip with the sampling noise, and with it the traversal mode)
constexpr double kPacketOffUtil = 0.3;
constexpr unsigned long long kPacketProbeFrames = 32;

void update_packet_choice(pgrt_ctx* ctx, const std::vector<FrameCounters>& fcs, int levels) {
    if (ctx->cfg.packet_levels != PGRT_PACKETS_AUTO) return;
    ctx->probe_level = -1;
    for (int L = 1; L < levels && L < kMaxLevels; ++L) {
        unsigned long long u = 0, l = 0;
        for (const FrameCounters& h : fcs) {
            u += h.pkt[L][0];
            l += h.pkt[L][1];
        }
        if (l < 4096) continue;  // not traced as packets (or too few rays to judge)
        ctx->packet_util[L] = (double)u / (double)l;
        if (ctx->packet_util[L] >= kPacketMinUtil) ctx->auto_packets |= 1u << L;
        else if (ctx->packet_util[L] < kPacketOffUtil) ctx->auto_packets &= ~(1u << L);
    }
    // re-probe the shallowest level that is off (its rays may have become coherent)
    if (++ctx->frames_collected % kPacketProbeFrames == 0)
        for (int L = 1; L < levels && L < kMaxLevels; ++L)
            if (!((ctx->auto_packets >> L) & 1u)) {
                ctx->probe_level = L;
                break;
            }
}

// 8-lanes-per-ray threshold: with frames in flight the concurrent frames hide the latency floors
// (r1 scan: 100k rays 0.392 -> 0.366 ms/frame), synchronous frames use the larger default
int group_max(const pgrt_ctx* ctx) {
    const int g = ctx->cfg.group_max;
    if (g < 0) return 0;
    if (g > 0) return g;
    return ctx->frames_in_flight > 1 ? kDefaultGroupMaxInFlight : kDefaultGroupMax;
}

// The tiles of each pipeline slot.  Round-robin (slot j gets tiles j, j + K, ...; multi-frame
// calls, tile-compact and distributed outputs rely on it: FrameParams::frame_tiles, store_pixel).
// A synchronous one-frame render into a framebuffer records which tiles' primary rays hit a
// dielectric (pgrt_config.tile_order) and, when the last frame of the same size had some, deals
// those tiles to slot 0 and the rest to slot 1: the frame's critical path is the chain of deep
// reflection / refraction levels (~20 dependent launches, each as long as its slowest ray), and
// it then starts after a level 0 over the deep tiles only, while slot 1's level 0 -- most of the
// pixels, no deep levels -- runs beside it.  Results do not depend on the deal (pixels are
// independent), only the schedule does.
std::vector<std::vector<int4>> deal_tiles(pgrt_ctx* ctx, FrameSet* fs, int K) {
    const std::vector<int4>& tiles = fs->tiles;
    std::vector<std::vector<int4>> deal(K);
    fs->deep_rec = K == 2 && fs->nframes == 1 && fs->out_mode == 0 && !fs->distributed &&
                   ctx->cfg.tile_order == 0 && fs->params.mode == PGRT_MODE_WHITTED && fs->params.max_level > 0;
    if (fs->deep_rec && ctx->deep_w == fs->cam_w && ctx->deep_h == fs->cam_h && !ctx->deep_tiles.empty()) {
        const int tx = (fs->cam_w + kTile - 1) / kTile;
        for (const int4& t : tiles) {
            const size_t id = (size_t)(t.y / kTile) * (size_t)tx + (size_t)(t.x / kTile);
            const bool deep = t.x >= 0 && t.y >= 0 && id < ctx->deep_tiles.size() && ctx->deep_tiles[id] != 0;
            deal[deep ? 0 : 1].push_back(t);
        }
        // no deep tiles, or most of the frame: the round-robin halves are the better split
        if (!deal[0].empty() && 2 * deal[0].size() <= tiles.size()) return deal;
        deal[0].clear();
        deal[1].clear();
    }
    for (size_t t = 0; t < tiles.size(); ++t) deal[t % K].push_back(tiles[t]);
    return deal;
}

// first level evaluated as whole ray trees in one launch (pgrt_config.subtree_level, subtree.hip),
// -1 = one launch per level
// Default: from level kSubtreeLevelSmall for one-frame batches of scenes up to kPacketBigScene
// triangles (the synchronous frame: levels 3.. are a few ten thousand rays whose per-level
// launches each last as long as their slowest ray; r4l timeline 0.583-0.597 -> 0.563 ms), one
// launch per level otherwise (the subtree launch's 8 lanes per ray cost multi-frame calls
// throughput: r4h driver line 0.179 -> 0.209 ms/frame).
int subtree_first(const pgrt_ctx* ctx, const SceneView& view, const pgrt_render_params* p, bool small_batch) {
    const int k = ctx->cfg.subtree_level;
    if (k < 0 || p->mode != PGRT_MODE_WHITTED || !subtree_available(view)) return -1;
    if (k > 0) return k <= p->max_level ? k : -1;
    return small_batch && view.ntri <= kPacketBigScene && kSubtreeLevelSmall <= p->max_level ? kSubtreeLevelSmall : -1;
}

// step budget of the bounce levels' packet launches (pgrt_config.packet_budget)
// pgrt_config.call_order: level 0 of calls in flight in submission order -- by default for big
// scenes only (BVH far beyond the L2: concurrent level-0 launches share the MALL and each other's
// misses; r3ab A/B: C5 18.1 -> 16.9 ms/frame, while the avenger's C2 / C3 lose 7 % / 87 % when
// their small, cache-resident level 0 is serialised)
bool call_ordered(const pgrt_ctx* ctx, const SceneView& view) {
    const int c = ctx->cfg.call_order;
    return c == 1 || (c == 0 && view.ntri > kPacketBigScene);
}

// The default budget follows the batch size: a one-frame batch (its bounce levels ~220k, ~100k
// rays: a few waves per SIMD) is bound by its slowest waves, so they hand over early (r3f:
// one-frame level 1 576 -> 309 us at 256 steps, 181 us at 64); a batch of several frames (8 per
// call: level 1 ~1.7M rays, tens of waves per SIMD) keeps its waves on packets longer, where 8
// lanes per deferred ray would cost throughput.  Decided by the batch's level-0 rays, not by the
// slot's queue hints (those describe whatever batch the slot rendered last).  Whitted frames of
// scenes up to kPacketBigScene triangles only: C5's 10^6-triangle soup and the path tracer's
// diffuse bounces defer far more rays at 64 steps and lose 8-9 % (profiles/r3/ab_r3ak_small_budget.txt)
int packet_budget(const pgrt_ctx* ctx, bool small_batch) {
    const int b = ctx->cfg.packet_budget;
    if (b != 0) return b < 0 ? 0 : b;
    return small_batch ? kSmallBatchPacketBudget : kDefaultPacketBudget;
}

// AUTO's probe (kProbeRays): after level L's own trace, a side packet launch over its first rays
// samples the packet utilisation of a level that is off packets (unprofiled frames only)
void probe_side_launch(pgrt_ctx* ctx, const SceneView& view, FrameSlot* sl, FrameCounters* fcd, const TraceLaunch& tl,
                       hipStream_t s) {
    const int L = tl.level;
    if (ctx->cfg.packet_levels != PGRT_PACKETS_AUTO || L < 1 || L != ctx->probe_level || ctx->timer.on ||
        packet_level(ctx, L) || !trace_packets_available(view) || tl.max_count <= 0)
        return;
    sl->probe_hits.alloc(kProbeRays);
    sl->probe_defer.alloc(kProbeRays);
    TraceLaunch pr = tl;
    pr.hits = sl->probe_hits.p;
    pr.max_count = std::min(tl.max_count, kProbeRays);
    pr.expect = pr.max_count;
    pr.count = false;
    pr.packets = true;
    pr.gen = nullptr;
    pr.budget = kDefaultPacketBudget;  // AUTO samples default-budget launches (packet_budget)
    pr.pkt_util = fcd->pkt[L];
    pr.defer_list = sl->probe_defer.p;
    pr.defer_count = &fcd->probe_defer;
    pr.resume = false;
    launch_trace(view, pr, s);
}

// One sample batch of a PGRT_MODE_PATH frame (path.hip): raygen, then per bounce L the closest
// hits of the path queue, the bounce's shading, its shadow rays and their resolve; the finish
// sums each pixel's path accumulators (a resolved level 0) and writes the output like a Whitted
// frame.  Per-path state lives in the level node buffers: n_color[0] = accumulators,
// n_link[L] (as int) = path index, n_att[L] = throughput of bounce L's queue.
void enqueue_path_batch(pgrt_ctx* ctx, FrameSlot* sl, const SceneView& view, const FrameParams& fp,
                        const pgrt_render_params* p, const Queue* q, FrameCounters* fcd, int n0, const FrameOut& fo,
                        int npix, bool first, bool last, int bi, int& trace_launches) {
    hipStream_t s = sl->stream;
    const int levels = p->max_level + 1;
    int id = ctx->timer.begin(s, CAT_RAYGEN);
    launch_raygen(ctx->cam, fp, sl->tiles.p, q[0], n0, fcd, s);
    ctx->timer.end(s, id);
    debug_sync(s, "path raygen", 0, bi);
    const ShadowQueue sq{sl->s_ro.p, sl->s_rd.p, sl->s_hit.p, sl->s_contrib.p, sl->s_cap, nullptr};
    float4* acc = sl->n_color[0]->p;
    const int nl = std::max(1, view.nlight);
    for (int L = 0; L < levels; ++L) {
        Queue qc = q[L & 1], qn = q[(L + 1) & 1];
        const int maxc = L == 0 ? n0 : std::min(sl->q_cap, sl->level_cap[L]);
        qc.cap = maxc;
        qn.cap = std::min(sl->q_cap, L + 1 < levels ? sl->level_cap[L + 1] : sl->q_cap);
        const int ex = L == 0 ? n0 : sl->expect_count[L];
        TraceLaunch tl;
        tl.level = L;
        tl.ro = qc.ro;
        tl.rd = qc.rd;
        tl.hits = qc.hit;
        tl.count_dev = fc_count_ptr(fcd, L);
        tl.max_count = maxc;
        tl.expect = ex;
        tl.gstack = sl->gstack.p;
        tl.gstack_threads = kTraceGridThreads;
        tl.counters = fcd->trav[L];
        tl.count = p->profile >= 2;
        tl.packets = packet_level(ctx, L);
        tl.pkt_util = fcd->pkt[L];
        tl.budget = packet_budget(ctx, false);
        tl.defer_list = sl->q_defer.p;
        tl.defer_count = &fcd->defer[L];
        tl.defer_expect = sl->expect_defer[L];
        id = ctx->timer.begin_kernel(CAT_TRACE, CAT_LTRACE + L);
        const bool launched = launch_trace(view, tl, s);
        ctx->timer.end_kernel(s, id, launched);
        ++trace_launches;
        debug_sync(s, "path trace", L, bi);
        probe_side_launch(ctx, view, sl, fcd, tl, s);
        const PathState ps{L > 0 ? reinterpret_cast<const int*>(sl->n_link[L]->p) : nullptr,
                           L > 0 ? sl->n_att[L]->p : nullptr,
                           L + 1 < levels ? reinterpret_cast<int*>(sl->n_link[L + 1]->p) : nullptr,
                           L + 1 < levels ? sl->n_att[L + 1]->p : nullptr, acc};
        id = ctx->timer.begin(s, CAT_SHADE, CAT_LSHADE + L);
        launch_path_shade(view, fp, ctx->cam.width, sl->tiles.p, L, qc, qn, ps, sq, fcd, maxc, ex, s);
        ctx->timer.end(s, id);
        debug_sync(s, "path shade", L, bi);
        if (view.nlight > 0 && L < p->max_level) {  // this bounce's hard shadow rays
            TraceLaunch st;
            st.ro = sq.ro;
            st.rd = sq.rd;
            st.hits = sq.hit;
            st.count_dev = fc_shadow_counts(fcd) + 2 * L;
            st.max_count = sq.cap;
            st.expect = (int)std::min<long long>((long long)ex * nl, sq.cap);
            st.gstack = sl->gstack.p;
            st.gstack_threads = kTraceGridThreads;
            st.counters = fcd->trav[kMaxLevels];
            st.count = p->profile >= 2;
            st.allow_group = false;
            id = ctx->timer.begin_kernel(CAT_TRACE, CAT_SHADOW);
            const bool sl_launched = launch_trace(view, st, s);
            ctx->timer.end_kernel(s, id, sl_launched);
            ++trace_launches;
            debug_sync(s, "path shadow trace", L, bi);
            id = ctx->timer.begin(s, CAT_COMBINE);
            launch_path_resolve(view, L, sq, ps, fcd, sq.cap, st.expect, s);
            ctx->timer.end(s, id);
            debug_sync(s, "path resolve", L, bi);
        }
    }
    id = ctx->timer.begin(s, CAT_COMBINE);
    launch_finish(view, fp, sl->tiles.p, LevelNodes{acc, nullptr, nullptr}, acc, sq, sl->accum.p, fo, npix, first, last,
                  true, nullptr, s);
    ctx->timer.end(s, id);
    debug_sync(s, "path finish", 0, bi);
}

// Enqueue the frame described by fs (params, tiles, output) on fs's slot streams after
// fs->ev_ready.  Tiles are <= kTile x kTile; out_mode 0 writes a framebuffer (origin ox,oy, pitch
// in pixels), 1 tile-compact buffers.  No host synchronisation.
void enqueue_frame(pgrt_ctx* ctx, FrameSet* fs) {
    const pgrt_render_params* p = &fs->params;
    const std::vector<int4>& tiles = fs->tiles;
    const int ntiles = (int)tiles.size();
    const int spp = p->spp_side * p->spp_side;
    const int levels = p->max_level + 1;
    // pipeline slots: tiles dealt round-robin (slot j gets tiles j, j+K, ...); one slot per frame
    // when frames are in flight: the concurrent frames fill the CUs instead (r1 scan: 6 frames x
    // 1 slot 0.39 ms/frame, 3 frames x 2 slots 0.53)
    const int want_slots = ctx->frames_in_flight > 1 ? 1 : kDefaultSlots;
    const int K = ntiles == 0 ? 0 : std::max(1, std::min(want_slots, ntiles));
    SceneView view = ctx->view;
    view.group_max = group_max(ctx);
    const long long max_batch = batch_rays(ctx);
    // level-0 rays generated inside the packet traversal (no k_raygen launch, no 32-B/ray read in
    // the traversal); it stores them for the level-0 shade
    const bool fuse = packet_level(ctx, 0) && trace_packets_available(view);
    fs->K = K;
    fs->batches = 0;
    while ((int)fs->slots.size() < K) fs->slots.emplace_back(new FrameSlot(fs->slots.empty()));
    const std::vector<std::vector<int4>> deal = deal_tiles(ctx, fs, K);
    // launch timeline (pgrt_timeline_enable): every launch of this call stamps its waves into
    // fs->stamps, the slot ranges handed out by the launchers through the stamp log
    StampLog slog;
    fs->stamp_launches.clear();
    fs->stamp_used = 0;
    if (ctx->timeline_on) {
        fs->stamps.alloc((size_t)kStampWaves * 2);
        slog.dev = fs->stamps.p;
        slog.cap = kStampWaves;
        slog.launches = &fs->stamp_launches;
    }
    struct LogScope {  // the thread's log never outlives this call (exceptions included)
        LogScope(StampLog* l) { set_stamp_log(l); }
        ~LogScope() { set_stamp_log(nullptr); }
    } log_scope(ctx->timeline_on ? &slog : nullptr);
    ctx->timer.on = p->profile > 0;
    int trace_launches = 0;
    FrameParams fp0{};
    fp0.slots = K;
    fp0.frame_tiles = fs->nframes > 1 ? fs->frame_tiles : 0;
    fp0.frame_out_tiles = fs->frame_out_tiles;
    fp0.frame_stride = fs->frame_stride;
    fp0.spp_side = p->spp_side;
    fp0.inv_s = 1.0f / (float)p->spp_side;
    fp0.jit_a = -0.5f / (float)p->spp_side;
    fp0.jit_b = 0.5f / (float)p->spp_side;
    fp0.max_level = p->max_level;
    fp0.dof = p->dof;
    fp0.focal = p->focal_distance;
    fp0.aperture = p->aperture;
    fp0.gamma = p->gamma_level;
    fp0.jitter = p->jitter;
    fp0.seed = p->seed;
    fp0.frame = p->frame;
    fp0.count = p->profile >= 2 ? 1 : 0;
    for (int j = 0; j < K; ++j) {
        FrameSlot* sl = fs->slots[j].get();
        hipStream_t s = sl->stream;
        slog.slot = j;
        const int nt = (int)deal[j].size();
        const long long npix = (long long)nt * kTile * kTile;
        const int nsb = (int)std::max(1ll, std::min<long long>(spp, max_batch / npix));
        PGRT_REQUIRE(npix * nsb < (1ll << 30), PGRT_ERR_INVALID_ARGUMENT,
                     "frame too large: " + std::to_string(npix) + " pixels in one pipeline slot");
        const int batches = (spp + nsb - 1) / nsb;
        fs->batches += batches;
        ensure_frame_buffers(sl, (int)(npix * nsb), levels, view.nlight, batches);
        sl->ensure_pinned(batches, nt);
        if (sl->tiles.n < (size_t)nt) sl->tiles_dev.clear();
        sl->tiles.alloc(nt);
        sl->accum.alloc((size_t)npix);
        PGRT_HIP(hipStreamWaitEvent(s, fs->ev_ready, 0));
        // the pinned tile list may still feed this slot's previous upload
        PGRT_HIP(hipEventSynchronize(sl->ev_done));
        std::copy(deal[j].begin(), deal[j].end(), sl->pinned_tiles);
        if (fs->deep_rec) sl->ensure_deep(nt, s);
        // the device tile list is re-uploaded only when it changed
        if (sl->tiles_dev.size() != (size_t)nt || !std::equal(sl->tiles_dev.begin(), sl->tiles_dev.end(),
                                                               sl->pinned_tiles, [](const int4& a, const int4& b) {
                                                                   return a.x == b.x && a.y == b.y && a.z == b.z &&
                                                                          a.w == b.w;
                                                               })) {
            PGRT_HIP(hipMemcpyAsync(sl->tiles.p, sl->pinned_tiles, sizeof(int4) * nt, hipMemcpyHostToDevice, s));
            sl->tiles_dev.assign(sl->pinned_tiles, sl->pinned_tiles + nt);
        }
        FrameParams fp = fp0;
        fp.ntiles = nt;
        fp.slot = j;
        fp.tile_deep = fs->deep_rec ? sl->tile_deep.p : nullptr;
        for (int bi = 0; bi < batches; ++bi) {
            const int s0 = bi * nsb;
            fp.s0 = s0;
            fp.nsb = std::min(nsb, spp - s0);
            const int n0 = (int)(npix * fp.nsb);
            FrameCounters* fcd = sl->fc.p + bi;
            Queue q[2];
            for (int b = 0; b < 2; ++b)
                q[b] = Queue{sl->q_ro[b].p, sl->q_rd[b].p, sl->q_time[b].p, sl->q_hit[b].p, sl->q_cap};
            // one light over the binary BVH: the compact shadow queue (no origins, one "lit" byte
            // per ray instead of a hit record: 47 B per shadow ray written and read fewer)
            const bool compact_shadow = view.nlight == 1 && !view.wide;
            ShadowQueue sq{compact_shadow ? nullptr : sl->s_ro.p, sl->s_rd.p, compact_shadow ? nullptr : sl->s_hit.p,
                           sl->s_contrib.p, sl->s_cap, compact_shadow ? sl->s_lit.p : nullptr};
            // pinhole level 0: the traversal stores directions only (the shade takes the origin,
            // tnear and medium from the camera: 20 B per primary ray written and read fewer)
            const bool dir_only = fuse && !p->dof;
            // one sample per pixel: a pixel whose primary ray misses is finished by the level-0
            // shade (L0Final), the finish completes the others
            const bool l0final = fuse && spp == 1;
            const FrameOut fo{fs->out, fs->out_mode, fs->ox, fs->oy, fs->pitch, K, j};
            if (p->mode == PGRT_MODE_PATH) {
                enqueue_path_batch(ctx, sl, view, fp, p, q, fcd, n0, fo, (int)npix, s0 == 0, s0 + fp.nsb >= spp, bi,
                                   trace_launches);
                continue;
            }
            const L0Final l0f{l0final ? sl->l0_hit.p : nullptr, l0final ? sl->l0_pending.p : nullptr, fo,
                              sl->tiles.p};
            const PrimaryGen gen{ctx->cam, fp, sl->tiles.p, dir_only ? nullptr : q[0].ro, q[0].rd,
                                 dir_only ? nullptr : q[0].time, &fcd->count0, l0f.hit};
            int id = ctx->timer.begin(s, CAT_RAYGEN);
            if (!fuse) launch_raygen(ctx->cam, fp, sl->tiles.p, q[0], n0, fcd, s);
            debug_sync(s, "raygen", 0, bi);
            ctx->timer.end(s, id);
            // levels >= sub: whole ray trees in one launch (no queues, shades or combines below it)
            const int sub = subtree_first(ctx, view, p, n0 < kSmallPacketBatch);
            for (int L = 0; L < levels; ++L) {
                Queue qc = q[L & 1], qn = q[(L + 1) & 1];
                const int maxc = L == 0 ? n0 : std::min(sl->q_cap, sl->level_cap[L]);
                qc.cap = maxc;
                qn.cap = std::min(sl->q_cap, L + 1 < levels ? sl->level_cap[L + 1] : sl->q_cap);
                LevelNodes ln{sl->n_color[L]->p, sl->n_link[L]->p, sl->n_att[L]->p};
                // grid hints: last frame's per-level counts (+25 %); level 0 is exact
                const int ex = L == 0 ? n0 : sl->expect_count[L];
                if (L == sub) {
                    id = ctx->timer.begin(s, CAT_TRACE, CAT_LTRACE + L);
                    launch_subtree(view, fp, L, qc, ln, fcd, maxc, ex, p->profile >= 2, s);
                    ctx->timer.end(s, id);
                    debug_sync(s, "subtree", L, bi);
                    ++trace_launches;
                    break;
                }
                TraceLaunch tl;
                tl.level = L;
                tl.ro = qc.ro;
                tl.rd = qc.rd;
                tl.hits = qc.hit;
                tl.count_dev = L == 0 && fuse ? nullptr : fc_count_ptr(fcd, L);
                tl.count_host = L == 0 && fuse ? n0 : 0;
                tl.max_count = maxc;
                tl.expect = ex;
                tl.gstack = sl->gstack.p;
                tl.gstack_threads = kTraceGridThreads;
                tl.counters = fcd->trav[L];
                tl.count = p->profile >= 2;
                tl.packets = packet_level(ctx, L);  // coherent 8x8-pixel waves -> packet traversal
                tl.gen = L == 0 && fuse ? &gen : nullptr;
                tl.budget = packet_budget(ctx, n0 < kSmallPacketBatch && view.ntri <= kPacketBigScene);
                // AUTO samples the packet utilisation of default-budget launches only: a wave cut
                // short at 64 steps reads as better used than it is, and one-frame batches would
                // then switch levels to packets for the multi-frame calls too
                tl.pkt_util = tl.budget == kSmallBatchPacketBudget && ctx->cfg.packet_budget == 0 ? nullptr : fcd->pkt[L];
                tl.defer_list = sl->q_defer.p;
                tl.defer_count = &fcd->defer[L];
                tl.defer_expect = sl->expect_defer[L];
                const bool ordered = L == 0 && K == 1 && ctx->frames_in_flight > 1 && call_ordered(ctx, view);
                if (ordered && ctx->l0_token_live) PGRT_HIP(hipStreamWaitEvent(s, ctx->l0_token, 0));
                id = ctx->timer.begin_kernel(CAT_TRACE, CAT_LTRACE + L);
                const bool launched = launch_trace(view, tl, s);
                ctx->timer.end_kernel(s, id, launched);
                debug_sync(s, "trace", L, bi);
                ++trace_launches;
                probe_side_launch(ctx, view, sl, fcd, tl, s);
                id = ctx->timer.begin(s, CAT_SHADE, CAT_LSHADE + L);
                const PinholeOrigin l0{ctx->cam.from[0], ctx->cam.from[1], ctx->cam.from[2], L == 0 && dir_only ? 1 : 0};
                launch_shade(view, fp, L, qc, qn, ln, sq, fcd, maxc, s, ex, l0,
                             L == 0 ? l0f : L0Final{nullptr, nullptr, fo, nullptr});
                debug_sync(s, "shade", L, bi);
                ctx->timer.end(s, id);
                if (ordered) {
                    if (!ctx->l0_token) PGRT_HIP(hipEventCreateWithFlags(&ctx->l0_token, hipEventDisableTiming));
                    PGRT_HIP(hipEventRecord(ctx->l0_token, s));
                    ctx->l0_token_live = true;
                }
            }
            if (view.nlight > 0 && p->max_level > 0) {  // every level's shadow rays, one launch
                TraceLaunch tl;
                tl.ro = sq.ro;
                tl.rd = sq.rd;
                tl.hits = sq.hit;
                tl.count_dev = fc_shadow_counts(fcd);
                tl.count_terms = sub > 0 ? sub : levels;  // the subtree levels trace their own shadow rays
                tl.max_count = sq.cap;
                tl.expect = sl->expect_shadow_total;
                tl.gstack = sl->gstack.p;
                tl.gstack_threads = kTraceGridThreads;
                tl.counters = fcd->trav[kMaxLevels];
                tl.count = p->profile >= 2;
                tl.allow_group = false;  // shadow rays: one lane per ray (no 8-lane groups, no packets)
                if (compact_shadow) {
                    tl.const_org = make_float4(ctx->light0[0], ctx->light0[1], ctx->light0[2], 0.01f);
                    tl.lit = sq.lit;
                }
                id = ctx->timer.begin_kernel(CAT_TRACE, CAT_SHADOW);
                const bool launched = launch_trace(view, tl, s);
                ctx->timer.end_kernel(s, id, launched);
                debug_sync(s, "shadow trace", levels, bi);
                ++trace_launches;
            }
            id = ctx->timer.begin(s, CAT_COMBINE);
            for (int L = std::min(p->max_level, sub > 0 ? sub : p->max_level) - 1; L >= 1; --L) {
                LevelNodes ln{sl->n_color[L]->p, sl->n_link[L]->p, sl->n_att[L]->p};
                launch_combine(view, L, ln, sl->n_color[L + 1]->p, sq, fcd, std::min(sl->q_cap, sl->level_cap[L]),
                               s, sl->expect_count[L]);
            }
            LevelNodes l0{sl->n_color[0]->p, sl->n_link[0]->p, sl->n_att[0]->p};
            const bool resolve_l0 = fp.nsb > 1;  // several samples per pixel: trees in parallel
            if (resolve_l0)
                launch_combine(view, 0, l0, levels > 1 ? sl->n_color[1]->p : sl->n_color[0]->p, sq, fcd, n0, s,
                               n0);
            debug_sync(s, "combine", 0, bi);
            launch_finish(view, fp, sl->tiles.p, l0, levels > 1 ? sl->n_color[1]->p : sl->n_color[0]->p, sq,
                          sl->accum.p, fo, (int)npix, s0 == 0, s0 + fp.nsb >= spp, resolve_l0, l0f.pending, s);
            debug_sync(s, "finish", 0, bi);
            ctx->timer.end(s, id);
        }
        sl->host_fc.resize(batches);
        // the frame's counters to pinned host memory, zeroed on the device for the next frame
        launch_export_counters(sl->fc.p, sl->pinned_fc, batches, fs->deep_rec ? sl->tile_deep.p : nullptr,
                               sl->pinned_deep, nt, s);
        debug_sync(s, "export", 0, 0);
        PGRT_HIP(hipEventRecord(sl->ev_done, s));
    }
    if (fs->host_dst && K > 0) {  // host output: after every slot, on slot 0's stream
        FrameSlot* s0 = fs->slots[0].get();
        for (int j = 1; j < K; ++j) PGRT_HIP(hipStreamWaitEvent(s0->stream, fs->slots[j]->ev_done, 0));
        PGRT_HIP(hipMemcpyAsync(fs->host_dst, fs->host_stage.p, fs->host_bytes, hipMemcpyDeviceToHost, s0->stream));
        PGRT_HIP(hipEventRecord(s0->ev_done, s0->stream));
    }
    PGRT_HIP(hipGetLastError());
    fs->stats.trace_launches = trace_launches;
    fs->stamp_used = slog.used;
}

// One look at fs's completed frame (host waits for its slots): the counters to the host, the next
// frame's grid hints.  Returns whether a queue of this rank overflowed (the frame is incomplete).
bool read_frame_counters(pgrt_ctx* ctx, FrameSet* fs) {
    const int K = fs->K;
    for (int j = 0; j < K; ++j) {
        FrameSlot* sl = fs->slots[j].get();
        PGRT_HIP(hipEventSynchronize(sl->ev_done));
        std::copy(sl->pinned_fc, sl->pinned_fc + sl->host_fc.size(), sl->host_fc.begin());
    }
    PGRT_HIP(hipGetLastError());
    if (fs->deep_rec) {  // pgrt_config.tile_order: the deep tiles of this frame for the next deal
        const int tx = (fs->cam_w + kTile - 1) / kTile, ty = (fs->cam_h + kTile - 1) / kTile;
        ctx->deep_tiles.assign((size_t)tx * ty, 0);
        ctx->deep_w = fs->cam_w;
        ctx->deep_h = fs->cam_h;
        for (int j = 0; j < K; ++j) {
            const FrameSlot* sl = fs->slots[j].get();
            for (size_t q = 0; q < sl->tiles_dev.size() && (int)q < sl->pinned_deep_n; ++q) {
                const int4 t = sl->tiles_dev[q];
                const size_t id = (size_t)(t.y / kTile) * (size_t)tx + (size_t)(t.x / kTile);
                if (t.x >= 0 && t.y >= 0 && id < ctx->deep_tiles.size() && sl->pinned_deep[q] != 0)
                    ctx->deep_tiles[id] = 1;
            }
        }
    }
    bool overflow = false;
    ctx->last_fc.clear();
    for (int j = 0; j < K; ++j) {
        FrameSlot* sl = fs->slots[j].get();
        for (auto& h : sl->host_fc) {
            overflow |= h.overflow != 0;
            ctx->last_fc.push_back(h);
        }
        int shadow_need = 0;
        for (auto& h : sl->host_fc) {
            int sc = 0;
            for (int L = 0; L < kMaxLevels; ++L) sc += fc_shadow(h, L);
            shadow_need = std::max(shadow_need, sc);
        }
        // grid hints for the next frame: kept while the count stays within [hint/2, hint]
        // (a stable hint keeps the captured launch sequence valid)
        auto hint = [](int& e, int c) {
            if (e == 0 || c > e || 2 * c + 2048 < e) e = c + c / 4 + 1024;
        };
        for (int L = 0; L < kMaxLevels; ++L) {
            int c = 0, dc = 0;
            for (auto& h : sl->host_fc) {
                c = std::max(c, fc_count(h, L));
                dc = std::max(dc, h.defer[L]);
            }
            hint(sl->expect_count[L], c);
            // deferral hints only from frames that deferred: a level traced without packets (AUTO
            // turned it off) defers nothing, and its next packet frame (a probe) needs the grid
            // its last packet frame needed, not the minimum
            if (dc > 0) hint(sl->expect_defer[L], dc);
        }
        hint(sl->expect_shadow_total, shadow_need);
    }
    return overflow;
}

// Re-render fs after a queue overflow: this rank's queues grow when it overflowed (grow), the
// timings of the failed attempt are dropped.
void rerender_frame(pgrt_ctx* ctx, FrameSet* fs, bool grow, int& retries) {
    const int levels = fs->params.max_level + 1;
    if (grow)
        for (int j = 0; j < fs->K; ++j) grow_after_overflow(fs->slots[j].get(), levels);
    double ms[CAT_N] = {0};
    ctx->timer.collect(ms);
    ++retries;
    PGRT_REQUIRE(retries < 8, PGRT_ERR_OUT_OF_MEMORY, "ray queues kept overflowing");
    enqueue_frame(ctx, fs);
}

// fs->stats of a complete frame (counters read by read_frame_counters); the context stream is
// then ordered after the frame.
void frame_stats(pgrt_ctx* ctx, FrameSet* fs, int retries) {
    const pgrt_render_params* p = &fs->params;
    const int levels = p->max_level + 1;
    const int spp = p->spp_side * p->spp_side;
    double ms[CAT_N] = {0};
    uint64_t rays_shadow = 0, rays_reflect = 0, rays_refract = 0, trav_nodes = 0, trav_tests = 0, trav_wide = 0;
    uint64_t shade_hits = 0, shade_textured = 0;
    update_packet_choice(ctx, ctx->last_fc, levels);
    for (auto& h : ctx->last_fc) {
        for (int L = 0; L < levels; ++L) {
            rays_shadow += (uint64_t)fc_shadow(h, L);
            if (L >= 1) {
                rays_refract += (uint64_t)h.refract[L];
                rays_reflect += (uint64_t)(fc_count(h, L) - h.refract[L]);
            }
        }
        for (int L = 0; L < kMaxLevels; ++L) {
            shade_hits += h.shade[L][0];
            shade_textured += h.shade[L][1];
        }
        for (int k = 0; k < 2 * kMaxLevels; ++k) {
            trav_wide += h.trav[k][14];
            trav_nodes += h.trav[k][0];
            trav_tests += h.trav[k][1];
        }
    }
    for (int j = 0; j < fs->K; ++j) PGRT_HIP(hipStreamWaitEvent(ctx->stream, fs->slots[j]->ev_done, 0));
    ctx->timer.collect(ms);
    pgrt_stats* st = &fs->stats;
    const int launches = st->trace_launches;
    *st = pgrt_stats{};
    long long real_pix = 0;
    for (auto& t : fs->tiles) real_pix += (long long)tile_width(t) * t.w;
    st->rays_primary = (uint64_t)(real_pix * spp);
    st->rays_shadow = rays_shadow;
    st->rays_reflect = rays_reflect;
    st->rays_refract = rays_refract;
    st->node_visits = trav_nodes;
    st->wide_node_visits = trav_wide;
    st->tri_tests = trav_tests;
    st->shade_hits = shade_hits;
    st->shade_textured_hits = shade_textured;
    st->ms_raygen = ms[CAT_RAYGEN];
    st->ms_trace = ms[CAT_TRACE];
    st->ms_shade = ms[CAT_SHADE];
    st->ms_shadow = ms[CAT_SHADOW];
    st->ms_combine = ms[CAT_COMBINE];
    for (int L = 0; L < kMaxLevels; ++L) {
        ctx->level_ms[L][0] = ms[CAT_LTRACE + L];
        ctx->level_ms[L][1] = ms[CAT_LSHADE + L];
    }
    st->trace_launches = launches;
    st->levels = levels;
    st->overflow_retries = retries;
    if (fs->stamp_used > 0 && fs->K > 0) {  // the call's launch timeline: (first wave start, last wave end) per launch
        ctx->stamp_host.resize((size_t)fs->stamp_used * 2);
        hipStream_t s0 = fs->slots[0]->stream;
        PGRT_HIP(hipMemcpyAsync(ctx->stamp_host.data(), fs->stamps.p, (size_t)fs->stamp_used * 16,
                                hipMemcpyDeviceToHost, s0));
        PGRT_HIP(hipStreamSynchronize(s0));
        std::vector<uint32_t> dur;
        for (const StampLaunch& l : fs->stamp_launches) {
            unsigned long long a = ~0ull, b = 0, last = 0;
            dur.clear();
            for (long long w = l.offset; w < l.offset + l.waves; ++w) {
                const unsigned long long t0 = ctx->stamp_host[2 * w], t1 = ctx->stamp_host[2 * w + 1];
                if (t0 == 0 || t1 < t0) continue;  // not a stamp of this launch
                a = std::min(a, t0);
                b = std::max(b, t1);
                last = std::max(last, t0);
                dur.push_back((uint32_t)std::min<unsigned long long>(t1 - t0, 0xffffffffull));
            }
            if (dur.empty()) continue;
            auto pct = [&](size_t q) {  // q-th percentile of the wave durations
                const size_t k = std::min(dur.size() - 1, dur.size() * q / 100);
                std::nth_element(dur.begin(), dur.begin() + k, dur.end());
                return dur[k];
            };
            pgrt_timeline_rec r{fs->ticket, l.slot, l.kind, l.level, (int)dur.size(), a, b, 0, 0, 0, 0};
            r.wave_p50 = pct(50);
            r.wave_p90 = pct(90);
            r.wave_max = *std::max_element(dur.begin(), dur.end());
            r.last_in = (uint32_t)(last - a);
            ctx->timeline.push_back(r);
        }
        fs->stamp_used = 0;
    }
}

void gather_frame(pgrt_ctx* ctx, FrameSet* fs);
void regather_rank0(pgrt_ctx* ctx, FrameSet* fs, bool own, const std::vector<int>& peers);

// a multi-process distributed frame whose gather goes over RCCL (the overflow flags ride along)
bool rccl_gather(const pgrt_ctx* ctx, const FrameSet* fs) {
    return fs->distributed && !ctx->emulated && fs->deal.world > 1 && ctx->comm != nullptr;
}

// Wait for fs's frame, re-render it after a queue overflow (larger queues), fill fs->stats.  A
// distributed frame's gather was queued with the frame (device-ordered, start_frame).  There is no
// control collective: a rank whose queues overflowed re-renders its tiles and sends them again;
// rank 0 learns which ranks did from the flag at the tail of every rank's send (gather_end copies
// them to host memory behind the unpack), receives those ranks' tiles again and unpacks them (and
// its own, when it overflowed).  Every rank posts its sends / receives for a frame when that frame
// is collected, and frames are collected in submission order on every rank, so the point-to-point
// operations stay matched.  Non-zero ranks never wait for another rank; rank 0 waits for the
// frame's own gather only.
void collect_frame(pgrt_ctx* ctx, FrameSet* fs) {
    int retries = 0;
    const bool rccl = rccl_gather(ctx, fs);
    for (;;) {
        const bool mine = read_frame_counters(ctx, fs);
        if (!rccl || ctx->rank != 0) {
            if (!mine) break;
            rerender_frame(ctx, fs, true, retries);
            if (fs->distributed) gather_frame(ctx, fs);  // rank != 0: the tiles again, to rank 0
            continue;
        }
        PGRT_HIP(hipEventSynchronize(fs->ev_flags));
        std::vector<int> peers;
        for (int r = 1; r < fs->deal.world; ++r)
            if (fs->peer_flags[r]) peers.push_back(r);
        if (!mine && peers.empty()) break;
        if (mine) {
            rerender_frame(ctx, fs, true, retries);
        } else {
            PGRT_REQUIRE(++retries < 8, PGRT_ERR_OUT_OF_MEMORY, "ray queues kept overflowing");
        }
        regather_rank0(ctx, fs, mine, peers);
    }
    frame_stats(ctx, fs, retries);
}

// this rank's tile count and every rank's list layout for a distributed frame of W x H
UnpackSrc unpack_layout(const TileDeal& d, int W, int H) {
    const int total = ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
    PGRT_REQUIRE(d.world >= 1 && d.world <= kMaxRanks, PGRT_ERR_INVALID_ARGUMENT,
                 "world size must be in [1, " + std::to_string(kMaxRanks) + "]");
    UnpackSrc u{};
    u.prefix[0] = 0;
    for (int r = 0; r < d.world; ++r) {
        u.count[r] = deal_count(d, total, r);
        u.prefix[r + 1] = u.prefix[r] + u.count[r];
    }
    return u;
}

// Distributed frame: every rank's tile-compact RGB buffer to rank 0 (grouped ncclSend / ncclRecv
// with each rank's exact tile count -- no padding crosses xGMI; rank 0's own tiles stay in place)
// and the unpack kernel there, on the context stream.  Queued when the frame is submitted: the
// context stream waits for the frame's slots on the DEVICE (hipStreamWaitEvent), so no rank's
// send, and neither rank 0's receive nor its unpack, waits for the host to see the frame done.
// Three parts, so a single-process multi-device context can put every rank's sends / receives
// in ONE ncclGroupStart / ncclGroupEnd (gather_begin, gather_post in a group, gather_end).
void gather_begin(pgrt_ctx* ctx, FrameSet* fs, UnpackSrc& u) {
    u = unpack_layout(fs->deal, fs->cam_w, fs->cam_h);
    for (int j = 0; j < fs->K; ++j) PGRT_HIP(hipStreamWaitEvent(ctx->stream, fs->slots[j]->ev_done, 0));
    PGRT_HIP(hipEventRecord(fs->ev_g0, ctx->stream));
    if (!ctx->emulated && fs->deal.world > 1 && ctx->comm) {
        // this rank's overflow flag after its tiles (the tail of its send): the exported counters
        FlagSrc f{};
        f.K = std::min(fs->K, 4);
        for (int j = 0; j < f.K; ++j) {
            f.fc[j] = fs->slots[j]->pinned_fc;
            f.n[j] = (int)fs->slots[j]->host_fc.size();
        }
        const size_t tiles = (size_t)fs->nframes * u.count[ctx->rank] * kTile * kTile * 3;
        launch_overflow_flag(f, reinterpret_cast<int*>(fs->tilebuf.p + tiles), ctx->stream);
    }
}

void gather_post(pgrt_ctx* ctx, FrameSet* fs, UnpackSrc& u) {
    const TileDeal& d = fs->deal;
    const int F = fs->nframes;
    const size_t tile_floats = (size_t)kTile * kTile * 3;  // RGB tiles (out_mode 2)
    const int me = ctx->rank;
    if (ctx->emulated) {
        // one GPU measures rank `me`: its tiles are copied to their place in a full-size buffer
        // (the other ranks' blocks stay unwritten), rank 0 also unpacks the whole frame
        ctx->gathered.alloc((size_t)F * u.prefix[d.world] * tile_floats);
        PGRT_HIP(hipMemcpyAsync(ctx->gathered.p + (size_t)F * u.prefix[me] * tile_floats, fs->tilebuf.p,
                                sizeof(float) * F * u.count[me] * tile_floats, hipMemcpyDeviceToDevice, ctx->stream));
        for (int r = 0; r < d.world; ++r) u.src[r] = ctx->gathered.p + (size_t)F * u.prefix[r] * tile_floats;
        return;
    }
    if (d.world == 1) {
        u.src[0] = fs->tilebuf.p;
        return;
    }
    PGRT_REQUIRE(ctx->comm, PGRT_ERR_RCCL, "pgrt_comm_init has not been called");
    auto ok = [](ncclResult_t r, const char* what) {
        if (r != ncclSuccess) throw Error(PGRT_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
    };
    // every rank's send: its tiles, then kGatherTail floats (the overflow flag, gather_begin)
    if (me == 0) {
        const size_t others = (size_t)F * (u.prefix[d.world] - u.count[0]) * tile_floats + (size_t)kGatherTail * (d.world - 1);
        ctx->gathered.alloc(std::max<size_t>(1, others));
        for (int r = 1; r < d.world; ++r) {
            float* dst = ctx->gathered.p + (size_t)F * (u.prefix[r] - u.count[0]) * tile_floats + (size_t)kGatherTail * (r - 1);
            u.src[r] = dst;
            if (!fs->regather || fs->regather_peer[r])
                ok(ncclRecv(dst, (size_t)F * u.count[r] * tile_floats + kGatherTail, ncclFloat, r, ctx->comm, ctx->stream),
                   "ncclRecv");
        }
        u.src[0] = fs->tilebuf.p;
    } else {
        ok(ncclSend(fs->tilebuf.p, (size_t)F * u.count[me] * tile_floats + kGatherTail, ncclFloat, 0, ctx->comm,
                    ctx->stream),
           "ncclSend");
    }
}

void gather_end(pgrt_ctx* ctx, FrameSet* fs, const UnpackSrc& u_in) {
    PGRT_HIP(hipEventRecord(fs->ev_g1, ctx->stream));
    UnpackSrc u = u_in;
    if (fs->regather)  // a re-gather: only the re-rendered ranks' tiles (the others' were unpacked already)
        for (int r = 0; r < fs->deal.world; ++r)
            if (!fs->regather_peer[r]) u.src[r] = nullptr;
    if (ctx->rank == 0)  // every frame of the call in one launch (grid.y = frame)
        launch_unpack_tiles(u, fs->dist_fb, fs->cam_w, fs->cam_h, fs->deal, 3, ctx->stream, 0, fs->nframes);
    if (ctx->rank == 0 && rccl_gather(ctx, fs) && !ctx->group) {  // the peers' overflow flags -> host
        launch_peer_flags(u, fs->deal.world, (size_t)fs->nframes * kTile * kTile * 3, fs->peer_flags, ctx->stream);
        PGRT_HIP(hipEventRecord(fs->ev_flags, ctx->stream));
    }
    PGRT_HIP(hipEventRecord(fs->ev_g2, ctx->stream));
    // the set's next frame overwrites its tile buffer only after the gather has read it
    PGRT_HIP(hipEventRecord(fs->ev_ready, ctx->stream));
    fs->gather_timed = true;
    PGRT_HIP(hipGetLastError());
}

void gather_frame(pgrt_ctx* ctx, FrameSet* fs) {
    UnpackSrc u;
    gather_begin(ctx, fs, u);
    auto ok = [](ncclResult_t r, const char* what) {
        if (r != ncclSuccess) throw Error(PGRT_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
    };
    const bool group = !ctx->emulated && fs->deal.world > 1;
    if (group) ok(ncclGroupStart(), "ncclGroupStart");  // one group for all of the call's frames
    gather_post(ctx, fs, u);
    if (group) ok(ncclGroupEnd(), "ncclGroupEnd");
    gather_end(ctx, fs, u);
}

// rank 0 after an overflow: receive the re-rendered tiles of `peers` again (their re-sends) and
// unpack those ranks' tiles, and its own when own (re-rendered in place)
void regather_rank0(pgrt_ctx* ctx, FrameSet* fs, bool own, const std::vector<int>& peers) {
    fs->regather = true;
    std::fill(fs->regather_peer, fs->regather_peer + kMaxRanks, 0);
    fs->regather_peer[0] = own ? 1 : 0;
    for (int r : peers) fs->regather_peer[r] = 1;
    std::fill(fs->peer_flags, fs->peer_flags + kMaxRanks, 0);
    try {
        gather_frame(ctx, fs);
    } catch (...) {
        fs->regather = false;
        throw;
    }
    fs->regather = false;
}

// device ms of a completed frame's gather (ncclGather incl. the wait for peers) + unpack
void gather_times(FrameSet* fs, pgrt_stats* st) {
    if (!fs->gather_timed) return;
    float g = 0, u = 0;
    PGRT_HIP(hipEventElapsedTime(&g, fs->ev_g0, fs->ev_g1));
    PGRT_HIP(hipEventElapsedTime(&u, fs->ev_g1, fs->ev_g2));
    st->ms_gather = g + u;
    st->ms_resolve = u;
}

// complete a pending frame: collect, gather (distributed), release the set's buffers
void finish_frame(pgrt_ctx* ctx, FrameSet* fs) {
    fs->pending = false;
    collect_frame(ctx, fs);  // a distributed frame's gather was queued at submission
    PGRT_HIP(hipEventRecord(fs->ev_ready, ctx->stream));
    fs->has_result = true;
    fs->stats.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - fs->t0).count();
}

void group_finish_through(pgrt_ctx* head, unsigned long long last);

// finish every pending frame with ticket <= last, oldest first (distributed frames gather in
// submission order on every rank; a multi-device context finishes every rank's frame together)
void finish_through(pgrt_ctx* ctx, unsigned long long last) {
    if (ctx->group) {
        group_finish_through(ctx, last);
        return;
    }
    for (;;) {
        FrameSet* oldest = nullptr;
        for (auto& s : ctx->sets)
            if (s->pending && s->ticket <= last && (!oldest || s->ticket < oldest->ticket)) oldest = s.get();
        if (!oldest) return;
        finish_frame(ctx, oldest);
    }
}

void drain_frames(pgrt_ctx* ctx) { finish_through(ctx, ~0ull); }

void check_frame(const pgrt_ctx* ctx, const pgrt_render_params* p) {
    PGRT_REQUIRE(ctx->has_scene, PGRT_ERR_NO_SCENE, "pgrt_set_scene has not been called");
    PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
    PGRT_REQUIRE(p->spp_side >= 1 && p->spp_side <= 64, PGRT_ERR_INVALID_ARGUMENT, "spp_side must be in [1, 64]");
    PGRT_REQUIRE(p->max_level >= 0 && p->max_level <= kMaxLevels - 2, PGRT_ERR_INVALID_ARGUMENT,
                 "max_level must be in [0, 14]");
    PGRT_REQUIRE(p->mode == PGRT_MODE_WHITTED || p->mode == PGRT_MODE_PATH, PGRT_ERR_INVALID_ARGUMENT,
                 "mode must be PGRT_MODE_WHITTED or PGRT_MODE_PATH");
}

// Start a frame on set fs (its previous frame must be finished).  distributed: out is ignored,
// the tiles land in fs->tilebuf and finish_frame gathers them into fb (rank 0).
void start_frame(pgrt_ctx* ctx, FrameSet* fs, const pgrt_render_params* p, std::vector<int4> tiles, float* out,
                 int out_mode, int ox, int oy, int pitch, bool distributed, float* fb, int nframes = 1,
                 long long frame_stride = 0, TileDeal deal = TileDeal{1, 1, 1}, bool defer_gather = false) {
    check_frame(ctx, p);
    PGRT_REQUIRE(nframes >= 1 && nframes <= kMaxFramesPerCall, PGRT_ERR_INVALID_ARGUMENT,
                 "frames per call must be in [1, 64]");
    PGRT_REQUIRE(!fs->host_dst || (!distributed && out == fs->host_stage.p), PGRT_ERR_INVALID_ARGUMENT,
                 "internal: a host destination is set for a frame that does not render into the staging buffer");
    fs->t0 = std::chrono::steady_clock::now();
    fs->params = *p;
    fs->nframes = nframes;
    fs->frame_tiles = (int)tiles.size();
    fs->frame_out_tiles = (int)tiles.size();
    fs->frame_stride = frame_stride;
    fs->tiles.clear();
    for (int f = 0; f < nframes; ++f)  // each record carries its frame (frame_of_tile)
        for (const int4& t : tiles) fs->tiles.push_back(make_int4(t.x, t.y, t.z | (f << kTileFrameShift), t.w));
    fs->distributed = distributed;
    fs->dist_fb = fb;
    fs->cam_w = ctx->cam.width;
    fs->cam_h = ctx->cam.height;
    if (distributed) {
        // this rank's tiles of every frame, frame-major (the gather's layout, unpack_layout)
        fs->deal = deal;
        // + the overflow flag's tail (gather_begin / collect_frame)
        fs->tilebuf.alloc((size_t)nframes * tiles.size() * kTile * kTile * 3 + kGatherTail);
        fs->frame_out_tiles = (int)tiles.size();
        out = fs->tilebuf.p;
        out_mode = 2;
        ox = oy = pitch = 0;
    }
    fs->out = out;
    fs->out_mode = out_mode;
    fs->ox = ox;
    fs->oy = oy;
    fs->pitch = pitch;
    fs->has_result = false;
    fs->ticket = ctx->next_ticket++;
    fs->gather_timed = false;
    enqueue_frame(ctx, fs);
    fs->pending = true;
    // the gather follows the frame on the device (a multi-device context groups every rank's
    // gather itself: defer_gather)
    if (distributed && !defer_gather) gather_frame(ctx, fs);
}

// Synchronous render of `tiles` (pending asynchronous frames complete first).
void render_tiles(pgrt_ctx* ctx, const pgrt_render_params* p, const std::vector<int4>& tiles, float* out,
                  int out_mode, int ox, int oy, int pitch, pgrt_stats* st, int nframes = 1,
                  long long frame_stride = 0) {
    drain_frames(ctx);
    FrameSet* fs = frame_set(ctx, 0);
    fs->host_dst = nullptr;
    PGRT_HIP(hipEventRecord(fs->ev_ready, ctx->stream));  // prior context-stream work first
    start_frame(ctx, fs, p, tiles, out, out_mode, ox, oy, pitch, false, nullptr, nframes, frame_stride);
    finish_frame(ctx, fs);
    if (st) *st = fs->stats;
}

std::vector<int4> rect_tiles(int x0, int y0, int w, int h) {
    std::vector<int4> t;
    for (int ty = 0; ty < h; ty += kTile)
        for (int tx = 0; tx < w; tx += kTile)
            t.push_back(make_int4(x0 + tx, y0 + ty, std::min(kTile, w - tx), std::min(kTile, h - ty)));
    return t;
}

void frame_rect(const pgrt_ctx* ctx, const pgrt_render_params* p, int& x, int& y, int& w, int& h) {
    x = p->rect_x;
    y = p->rect_y;
    w = p->rect_w;
    h = p->rect_h;
    if (w <= 0 || h <= 0) {
        x = 0;
        y = 0;
        w = ctx->cam.width;
        h = ctx->cam.height;
    }
    PGRT_REQUIRE(x >= 0 && y >= 0 && x + w <= ctx->cam.width && y + h <= ctx->cam.height, PGRT_ERR_INVALID_ARGUMENT,
                 "render rect outside the camera image");
}

// the deal of this context's distributed frames (pgrt_config.rank0_share_*, else the default)
TileDeal ctx_deal(const pgrt_ctx* ctx, int world) {
    return tile_deal(world, ctx->cfg.rank0_share_a, ctx->cfg.rank0_share_b);
}

// rank's tiles in its local order (tiles.hpp deal)
std::vector<int4> rank_tiles(int W, int H, int rank, const TileDeal& d) {
    std::vector<int4> all = rect_tiles(0, 0, W, H), mine;
    for (int j = 0;; ++j) {
        const int t = deal_tile(d, rank, j);
        if (t >= (int)all.size()) break;
        mine.push_back(all[t]);
    }
    return mine;
}

// ---- single-process multi-device context (pgrt_create_devices) --------------------------
// One host thread drives every rank: each rank's frame is enqueued on its own device, the
// gathers of all ranks go into ONE ncclGroupStart / ncclGroupEnd (the form RCCL requires when
// one thread owns several communicators), and the queue-overflow agreement is a host OR over
// the ranks' counters (no control collective).  Every rank uses frame set (ticket mod frames in
// flight), so the ranks' sets stay in lockstep.

std::vector<pgrt_ctx*> group_ranks(pgrt_ctx* head) {
    std::vector<pgrt_ctx*> r{head};
    r.insert(r.end(), head->members.begin(), head->members.end());
    return r;
}

void on_device(const pgrt_ctx* c) { PGRT_HIP(hipSetDevice(c->device)); }

// every rank's gather of the frames on set si: grouped ncclSend / ncclRecv, or (ranks sharing a
// device) device copies into rank 0's gather buffer on rank 0's stream
void group_gather(const std::vector<pgrt_ctx*>& R, int si) {
    const size_t n = R.size();
    std::vector<UnpackSrc> u(n);
    for (size_t i = 0; i < n; ++i) {
        on_device(R[i]);
        gather_begin(R[i], frame_set(R[i], si), u[i]);
    }
    pgrt_ctx* head = R[0];
    FrameSet* h = frame_set(head, si);
    if (head->peer_copy && n > 1) {
        on_device(head);
        const TileDeal& d = h->deal;
        const size_t tile_floats = (size_t)kTile * kTile * 3;
        const size_t F = (size_t)h->nframes;
        UnpackSrc& u0 = u[0];
        head->gathered.alloc(std::max<size_t>(1, F * (u0.prefix[d.world] - u0.count[0]) * tile_floats));
        u0.src[0] = h->tilebuf.p;
        for (size_t r = 1; r < n; ++r) {
            FrameSet* m = frame_set(R[r], (int)si);
            float* dst = head->gathered.p + F * (u0.prefix[r] - u0.count[0]) * tile_floats;
            u0.src[r] = dst;
            // rank r's frame is complete when its gather_begin event is (it follows the slots)
            PGRT_HIP(hipStreamWaitEvent(head->stream, m->ev_g0, 0));
            if (u0.count[r] > 0)
                PGRT_HIP(hipMemcpyPeerAsync(dst, head->device, m->tilebuf.p, R[r]->device,
                                            sizeof(float) * F * u0.count[r] * tile_floats, head->stream));
        }
        gather_end(head, h, u0);
        for (size_t r = 1; r < n; ++r) {
            on_device(R[r]);
            // a member's next frame on this set overwrites its tile buffer after rank 0 copied it
            PGRT_HIP(hipStreamWaitEvent(R[r]->stream, h->ev_g1, 0));
            gather_end(R[r], frame_set(R[r], (int)si), u[r]);
        }
        return;
    }
    auto ok = [](ncclResult_t r, const char* what) {
        if (r != ncclSuccess) throw Error(PGRT_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
    };
    if (n > 1) ok(ncclGroupStart(), "ncclGroupStart");
    for (size_t i = 0; i < n; ++i) {
        on_device(R[i]);
        gather_post(R[i], frame_set(R[i], (int)si), u[i]);
    }
    if (n > 1) ok(ncclGroupEnd(), "ncclGroupEnd");
    for (size_t i = 0; i < n; ++i) {
        on_device(R[i]);
        gather_end(R[i], frame_set(R[i], (int)si), u[i]);
    }
}

// complete the frame on set si of every rank: counters, re-render + re-gather on any rank's
// overflow, stats; rank 0's stats describe the whole frame (counts summed over the ranks,
// device times of the slowest rank)
void group_finish_set(pgrt_ctx* head, int si) {
    const std::vector<pgrt_ctx*> R = group_ranks(head);
    std::vector<char> mine(R.size());
    int retries = 0;
    for (pgrt_ctx* m : R) frame_set(m, si)->pending = false;
    for (;;) {
        bool any = false;
        for (size_t i = 0; i < R.size(); ++i) {
            on_device(R[i]);
            mine[i] = read_frame_counters(R[i], frame_set(R[i], si));
            any |= mine[i] != 0;
        }
        if (!any) break;
        const int tries = retries;
        for (size_t i = 0; i < R.size(); ++i) {
            on_device(R[i]);
            int t = tries;
            rerender_frame(R[i], frame_set(R[i], si), mine[i] != 0, t);
            retries = t;
        }
        group_gather(R, si);
    }
    pgrt_stats sum{};
    for (size_t i = 0; i < R.size(); ++i) {
        on_device(R[i]);
        FrameSet* fs = frame_set(R[i], si);
        frame_stats(R[i], fs, retries);
        PGRT_HIP(hipEventRecord(fs->ev_ready, R[i]->stream));
        fs->has_result = true;
        const pgrt_stats& s = fs->stats;
        sum.rays_primary += s.rays_primary;
        sum.rays_shadow += s.rays_shadow;
        sum.rays_reflect += s.rays_reflect;
        sum.rays_refract += s.rays_refract;
        sum.node_visits += s.node_visits;
        sum.tri_tests += s.tri_tests;
        sum.wide_node_visits += s.wide_node_visits;
        sum.shade_hits += s.shade_hits;
        sum.shade_textured_hits += s.shade_textured_hits;
        sum.ms_raygen = std::max(sum.ms_raygen, s.ms_raygen);
        sum.ms_trace = std::max(sum.ms_trace, s.ms_trace);
        sum.ms_shade = std::max(sum.ms_shade, s.ms_shade);
        sum.ms_shadow = std::max(sum.ms_shadow, s.ms_shadow);
        sum.ms_combine = std::max(sum.ms_combine, s.ms_combine);
        sum.trace_launches = std::max(sum.trace_launches, s.trace_launches);
        sum.levels = std::max(sum.levels, s.levels);
    }
    on_device(head);
    FrameSet* h = frame_set(head, si);
    sum.overflow_retries = retries;
    h->stats = sum;
    h->stats.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h->t0).count();
}

void group_finish_through(pgrt_ctx* head, unsigned long long last) {
    for (;;) {
        int oldest = -1;
        for (int i = 0; i < (int)head->sets.size(); ++i) {
            const FrameSet* s = head->sets[i].get();
            if (s->pending && s->ticket <= last && (oldest < 0 || s->ticket < head->sets[oldest]->ticket)) oldest = i;
        }
        if (oldest < 0) break;
        group_finish_set(head, oldest);
    }
    on_device(head);
}

// enqueue nframes distributed frames on every rank (rank 0's output: fb, frame-major W x H
// RGBA) and their grouped gather; returns the ticket
unsigned long long group_submit(pgrt_ctx* head, const pgrt_render_params* p, int nframes, float* fb) {
    PGRT_REQUIRE(fb, PGRT_ERR_INVALID_ARGUMENT, "a multi-device context needs an output buffer");
    PGRT_REQUIRE(p->rect_w <= 0 || (p->rect_x == 0 && p->rect_y == 0 && p->rect_w == head->cam.width &&
                                     p->rect_h == head->cam.height),
                 PGRT_ERR_INVALID_ARGUMENT, "a multi-device context renders whole frames (no render rect)");
    const std::vector<pgrt_ctx*> R = group_ranks(head);
    const int si = (int)(head->next_ticket % (unsigned long long)head->frames_in_flight);
    FrameSet* h = frame_set(head, si);
    if (h->pending) group_finish_through(head, h->ticket);  // the set's previous frame first
    const TileDeal deal = ctx_deal(head, (int)R.size());
    const unsigned long long ticket = head->next_ticket;
    for (pgrt_ctx* m : R) {
        on_device(m);
        FrameSet* fs = frame_set(m, si);
        fs->host_dst = nullptr;
        m->next_ticket = ticket;  // every rank's frame carries rank 0's ticket
        start_frame(m, fs, p, rank_tiles(head->cam.width, head->cam.height, m->rank, deal), nullptr, 1, 0, 0, 0,
                    true, m == head ? fb : nullptr, nframes, 0, deal, true);
    }
    group_gather(R, si);
    on_device(head);
    return ticket;
}

// synchronous group frame(s) into fb (rank 0's device)
void group_render(pgrt_ctx* head, const pgrt_render_params* p, int nframes, float* fb, pgrt_stats* st) {
    group_finish_through(head, ~0ull);
    const unsigned long long t = group_submit(head, p, nframes, fb);
    group_finish_through(head, t);
    FrameSet* fs = nullptr;
    for (auto& s : head->sets)
        if (s->ticket == t) fs = s.get();
    PGRT_HIP(hipEventSynchronize(fs->ev_ready));
    gather_times(fs, &fs->stats);
    if (st) *st = fs->stats;
}

}  // namespace

// =========================================================================== C ABI

extern "C" {

const char* pgrt_version(void) { return "pgrt 0.1.0 (gfx950, abi 1)"; }

int pgrt_device_count(int* count) {
    if (!count) return PGRT_ERR_INVALID_ARGUMENT;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return PGRT_OK;
}

int pgrt_create(int hip_device, pgrt_ctx** out) {
    if (!out) return PGRT_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return PGRT_ERR_NO_DEVICE;
    if (hip_device < 0 || hip_device >= n) return PGRT_ERR_INVALID_ARGUMENT;
    pgrt_ctx* ctx = new (std::nothrow) pgrt_ctx();
    if (!ctx) return PGRT_ERR_OUT_OF_MEMORY;
    ctx->device = hip_device;
    if (const char* e = getenv("PGRT_EMULATE_RANK")) {
        int r = 0, w = 1;
        if (sscanf(e, "%d/%d", &r, &w) == 2 && w >= 1 && w <= kMaxRanks && r >= 0 && r < w) {
            ctx->world = w;
            ctx->rank = r;
            ctx->emulated = w > 1;
        }
    }
    int rc = guarded(ctx, [&] { PGRT_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)); });
    if (rc != PGRT_OK) {
        delete ctx;
        return rc;
    }
    *out = ctx;
    return PGRT_OK;
}

int pgrt_create_devices(const int* hip_device_ids, int n_devices, pgrt_ctx** out) {
    if (!out || !hip_device_ids || n_devices < 1 || n_devices > kMaxRanks) return PGRT_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    pgrt_ctx* head = nullptr;
    int rc = pgrt_create(hip_device_ids[0], &head);
    if (rc != PGRT_OK) return rc;
    for (int r = 1; r < n_devices; ++r) {
        pgrt_ctx* m = nullptr;
        rc = pgrt_create(hip_device_ids[r], &m);
        if (rc != PGRT_OK) {
            delete head;
            return rc;
        }
        head->members.push_back(m);
    }
    rc = guarded(head, [&] {
        const std::vector<pgrt_ctx*> R = group_ranks(head);
        bool distinct = true;
        for (int a = 0; a < n_devices; ++a)
            for (int b = 0; b < a; ++b) distinct &= hip_device_ids[a] != hip_device_ids[b];
        for (int r = 0; r < n_devices; ++r) {
            R[r]->world = n_devices;
            R[r]->rank = r;
            R[r]->emulated = false;
        }
        head->group = true;
        head->peer_copy = !distinct;
        if (distinct) {  // one communicator per device, all created by this thread
            std::vector<ncclComm_t> comms(n_devices, nullptr);
            const ncclResult_t r = ncclCommInitAll(comms.data(), n_devices, hip_device_ids);
            if (r != ncclSuccess) throw Error(PGRT_ERR_RCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
            for (int k = 0; k < n_devices; ++k) R[k]->comm = comms[k];
        }
    });
    if (rc != PGRT_OK) {
        delete head;
        return rc;
    }
    *out = head;
    return PGRT_OK;
}

void pgrt_destroy(pgrt_ctx* ctx) {
    if (!ctx) return;
    if (ctx->group) (void)guarded(ctx, [&] { drain_frames(ctx); });
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    delete ctx;
}

const char* pgrt_last_error(const pgrt_ctx* ctx) { return ctx ? ctx->err.c_str() : "NULL context"; }

int pgrt_get_config(const pgrt_ctx* ctx, pgrt_config* cfg) {
    if (!ctx || !cfg) return PGRT_ERR_INVALID_ARGUMENT;
    *cfg = ctx->cfg;
    return PGRT_OK;
}

int pgrt_set_config(pgrt_ctx* ctx, const pgrt_config* cfg) {
    if (!ctx || !cfg) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(cfg->bvh_builder == 0 || cfg->bvh_builder == PGRT_BVH_LBVH || cfg->bvh_builder == PGRT_BVH_PLOC,
                     PGRT_ERR_INVALID_ARGUMENT, "bvh_builder must be 0, PGRT_BVH_LBVH or PGRT_BVH_PLOC");
        PGRT_REQUIRE(cfg->bvh_width == 0 || cfg->bvh_width == 2 || cfg->bvh_width == 8, PGRT_ERR_INVALID_ARGUMENT,
                     "bvh_width must be 0, 2 or 8");
        PGRT_REQUIRE(cfg->split_beta >= 0.0f && cfg->split_beta <= 4.0f, PGRT_ERR_INVALID_ARGUMENT,
                     "split_beta must be in [0, 4]");
        PGRT_REQUIRE(cfg->packet_levels >= PGRT_PACKETS_OFF && cfg->packet_levels <= kMaxLevels,
                     PGRT_ERR_INVALID_ARGUMENT, "packet_levels must be AUTO, OFF or in [1, 16]");
        PGRT_REQUIRE(cfg->max_batch_rays >= 0 && cfg->max_batch_rays <= (1ll << 29), PGRT_ERR_INVALID_ARGUMENT,
                     "max_batch_rays must be in [0, 2^29]");
        PGRT_REQUIRE(cfg->max_batches_in_flight >= 0, PGRT_ERR_INVALID_ARGUMENT, "max_batches_in_flight must be >= 0");
        PGRT_REQUIRE(cfg->packet_budget >= -1, PGRT_ERR_INVALID_ARGUMENT,
                     "packet_budget must be -1 (off), 0 (default) or a step count");
        PGRT_REQUIRE(cfg->tile_order == 0 || cfg->tile_order == -1, PGRT_ERR_INVALID_ARGUMENT,
                     "tile_order must be 0 (default: deep tiles first) or -1 (round-robin)");
        PGRT_REQUIRE(cfg->call_order == 0 || cfg->call_order == 1 || cfg->call_order == -1, PGRT_ERR_INVALID_ARGUMENT,
                     "call_order must be 0 (default), 1 (level 0 in submission order) or -1 (free)");
        PGRT_REQUIRE(cfg->rank0_share_a >= 0 && cfg->rank0_share_a <= 64 && cfg->rank0_share_b >= 0 &&
                         cfg->rank0_share_b <= 64,
                     PGRT_ERR_INVALID_ARGUMENT, "rank0_share_a / rank0_share_b must be in [0, 64]");
        drain_frames(ctx);  // pending frames were enqueued with the old choices
        ctx->cfg = *cfg;
        for (pgrt_ctx* m : ctx->members) m->cfg = *cfg;  // a multi-device context: every rank
    });
}

int pgrt_set_scene(pgrt_ctx* ctx, const pgrt_scene_desc* scene) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        drain_frames(ctx);  // frames in flight read the old scene
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
        set_scene(ctx, scene);
        for (pgrt_ctx* m : ctx->members) {  // a multi-device context: the same build on every rank
            on_device(m);
            PGRT_HIP(hipStreamSynchronize(m->stream));
            set_scene(m, scene);
        }
    });
}

int pgrt_bvh_get_info(const pgrt_ctx* ctx, pgrt_bvh_info* info) {
    if (!ctx || !info) return PGRT_ERR_INVALID_ARGUMENT;
    if (!ctx->has_scene) return PGRT_ERR_NO_SCENE;
    *info = ctx->info;
    return PGRT_OK;
}

int pgrt_set_camera(pgrt_ctx* ctx, const pgrt_camera* cam) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(cam && cam->width > 0 && cam->height > 0 && cam->width <= 65536 && cam->height <= 65536,
                     PGRT_ERR_INVALID_ARGUMENT, "camera resolution must be in [1, 65536]");
        ctx->cam = make_camera(*cam);
        ctx->has_cam = true;
        for (pgrt_ctx* m : ctx->members) {
            m->cam = ctx->cam;
            m->has_cam = true;
        }
    });
}

int pgrt_render_device(pgrt_ctx* ctx, const pgrt_render_params* p, void* rgba_device, pgrt_stats* st) {
    if (!ctx || !p || !rgba_device) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        auto t0 = std::chrono::steady_clock::now();
        int x, y, w, h;
        frame_rect(ctx, p, x, y, w, h);
        if (ctx->group)  // every rank renders its tiles, rank 0 gathers (pgrt_create_devices)
            group_render(ctx, p, 1, static_cast<float*>(rgba_device), st);
        else
            render_tiles(ctx, p, rect_tiles(x, y, w, h), static_cast<float*>(rgba_device), 0, x, y, w, st);
        if (st) st->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

int pgrt_render_frames_device(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes, void* rgba_device,
                              pgrt_stats* st) {
    if (!ctx || !p || !rgba_device) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        auto t0 = std::chrono::steady_clock::now();
        int x, y, w, h;
        frame_rect(ctx, p, x, y, w, h);
        if (ctx->group)
            group_render(ctx, p, nframes, static_cast<float*>(rgba_device), st);
        else
            render_tiles(ctx, p, rect_tiles(x, y, w, h), static_cast<float*>(rgba_device), 0, x, y, w, st, nframes,
                         (long long)w * h * 4);
        if (st) st->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

int pgrt_render(pgrt_ctx* ctx, const pgrt_render_params* p, float* rgba_host, pgrt_stats* st) {
    if (!ctx || !p || !rgba_host) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        auto t0 = std::chrono::steady_clock::now();
        int x, y, w, h;
        frame_rect(ctx, p, x, y, w, h);
        ctx->out_tmp.alloc((size_t)w * h * 4);
        if (ctx->group)
            group_render(ctx, p, 1, ctx->out_tmp.p, st);
        else
            render_tiles(ctx, p, rect_tiles(x, y, w, h), ctx->out_tmp.p, 0, x, y, w, st);
        PGRT_HIP(hipMemcpyAsync(rgba_host, ctx->out_tmp.p, (size_t)w * h * 4 * sizeof(float), hipMemcpyDeviceToHost,
                                ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
        if (st) st->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

int pgrt_device_alloc(pgrt_ctx* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        hipError_t e = hipMalloc(out, bytes ? bytes : 1);
        if (e != hipSuccess) throw Error(PGRT_ERR_OUT_OF_MEMORY, hipGetErrorString(e));
    });
}

int pgrt_device_free(pgrt_ctx* ctx, void* ptr) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] { PGRT_HIP(hipFree(ptr)); });
}

int pgrt_copy_to_host(pgrt_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int pgrt_synchronize(pgrt_ctx* ctx) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        for (pgrt_ctx* m : ctx->members) {
            on_device(m);
            PGRT_HIP(hipStreamSynchronize(m->stream));
        }
        on_device(ctx);
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
    });
}

extern "C++" {
namespace {
// closest hits of n rays: ray(i, a, b) fills ray i's (org, tnear) / (dir, tfar); the hit records
// (t, u, v, prim bits) land in out (n float4, host)
template <class RayFn>
void intersect_rays(pgrt_ctx* ctx, int n, RayFn ray, float4* out) {
        DevBuf<float4> ro, rd, h;
        ro.alloc(n);
        rd.alloc(n);
        h.alloc(n);
        std::vector<float4> a(n), b(n);
        for (int i = 0; i < n; ++i) ray(i, a[i], b[i]);
        PGRT_HIP(hipMemcpyAsync(ro.p, a.data(), sizeof(float4) * n, hipMemcpyHostToDevice, ctx->stream));
        PGRT_HIP(hipMemcpyAsync(rd.p, b.data(), sizeof(float4) * n, hipMemcpyHostToDevice, ctx->stream));
        if (ctx->gstack.n == 0) ctx->gstack.alloc((size_t)kTraceGridThreads * kGlobalStack);
        TraceLaunch tl;
        tl.ro = ro.p;
        tl.rd = rd.p;
        tl.hits = h.p;
        tl.count_host = n;
        tl.max_count = n;
        tl.gstack = ctx->gstack.p;
        tl.gstack_threads = kTraceGridThreads;
        SceneView view = ctx->view;
        view.group_max = group_max(ctx);  // batches up to it: 8 / 4 lanes per ray
        launch_trace(view, tl, ctx->stream);
        PGRT_HIP(hipGetLastError());
        PGRT_HIP(hipMemcpyAsync(out, h.p, sizeof(float4) * n, hipMemcpyDeviceToHost, ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
}
}  // namespace
}  // extern "C++"

int pgrt_intersect_closest(pgrt_ctx* ctx, const float* rays, int n, float* hits) {
    if (!ctx || n < 0 || (n > 0 && (!rays || !hits))) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_scene, PGRT_ERR_NO_SCENE, "pgrt_set_scene has not been called");
        if (n == 0) return;
        intersect_rays(
            ctx, n,
            [&](int i, float4& a, float4& b) {
                const float* r = rays + 8 * (size_t)i;
                a = make_float4(r[0], r[1], r[2], r[3]);
                b = make_float4(r[4], r[5], r[6], r[7]);
            },
            reinterpret_cast<float4*>(hits));
    });
}

int pgrt_intersect_closest_soa(pgrt_ctx* ctx, const float* rays_soa, int n, float* hits_soa) {
    if (!ctx || n < 0 || (n > 0 && (!rays_soa || !hits_soa))) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_scene, PGRT_ERR_NO_SCENE, "pgrt_set_scene has not been called");
        if (n == 0) return;
        const size_t N = (size_t)n;
        std::vector<float4> h(N);
        intersect_rays(
            ctx, n,
            [&](int i, float4& a, float4& b) {
                const float* r = rays_soa + i;
                a = make_float4(r[0], r[N], r[2 * N], r[3 * N]);
                b = make_float4(r[4 * N], r[5 * N], r[6 * N], r[7 * N]);
            },
            h.data());
        for (size_t i = 0; i < N; ++i) {
            hits_soa[i] = h[i].x;
            hits_soa[N + i] = h[i].y;
            hits_soa[2 * N + i] = h[i].z;
            hits_soa[3 * N + i] = h[i].w;
        }
    });
}

int pgrt_occluded(pgrt_ctx* ctx, const float* rays, int n, int* occluded) {
    if (!ctx || n < 0 || (n > 0 && (!rays || !occluded))) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_scene, PGRT_ERR_NO_SCENE, "pgrt_set_scene has not been called");
        if (n == 0) return;
        DevBuf<float4> ro, rd;
        DevBuf<int> occ;
        ro.alloc(n);
        rd.alloc(n);
        occ.alloc(n);
        std::vector<float4> a(n), b(n);
        for (int i = 0; i < n; ++i) {
            const float* r = rays + 8 * (size_t)i;
            a[i] = make_float4(r[0], r[1], r[2], r[3]);
            b[i] = make_float4(r[4], r[5], r[6], r[7]);
        }
        PGRT_HIP(hipMemcpyAsync(ro.p, a.data(), sizeof(float4) * n, hipMemcpyHostToDevice, ctx->stream));
        PGRT_HIP(hipMemcpyAsync(rd.p, b.data(), sizeof(float4) * n, hipMemcpyHostToDevice, ctx->stream));
        launch_occluded(ctx->view, ro.p, rd.p, n, occ.p, ctx->stream);
        PGRT_HIP(hipGetLastError());
        PGRT_HIP(hipMemcpyAsync(occluded, occ.p, sizeof(int) * n, hipMemcpyDeviceToHost, ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
    });
}

// ---- frame sink: progressive accumulation ----------------------------------------------------

int pgrt_accumulate_reset(pgrt_ctx* ctx) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    ctx->acc_count = 0;
    return PGRT_OK;
}

int pgrt_render_accumulate(pgrt_ctx* ctx, const pgrt_render_params* p, float* mean_host, int* frames,
                           pgrt_stats* st) {
    if (!ctx || !p) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        auto t0 = std::chrono::steady_clock::now();
        int x, y, w, h;
        frame_rect(ctx, p, x, y, w, h);
        if (w != ctx->acc_w || h != ctx->acc_h) ctx->acc_count = 0;  // a new frame size restarts the sum
        const size_t px = (size_t)w * h;
        ctx->acc_frame.alloc(px * 4);
        ctx->acc_sum.alloc(px * 4);
        ctx->acc_mean.alloc(px * 4);
        render_tiles(ctx, p, rect_tiles(x, y, w, h), ctx->acc_frame.p, 0, x, y, w, st);
        ctx->acc_w = w;
        ctx->acc_h = h;
        ++ctx->acc_count;
        launch_accumulate_frame(ctx->acc_frame.p, ctx->acc_sum.p, ctx->acc_mean.p, (long long)px, ctx->acc_count,
                                ctx->stream);
        PGRT_HIP(hipGetLastError());
        if (mean_host)
            PGRT_HIP(hipMemcpyAsync(mean_host, ctx->acc_mean.p, px * 4 * sizeof(float), hipMemcpyDeviceToHost,
                                    ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
        if (frames) *frames = ctx->acc_count;
        if (st) st->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

// ---- tiles / multi-GPU -------------------------------------------------------------------

int pgrt_tile_count_ex(int width, int height, int tile_size, int rank, int world, int a, int b) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || world <= 0 || rank < 0 || rank >= world || a < 0 || b < 0 ||
        a > 64 || b > 64)
        return PGRT_ERR_INVALID_ARGUMENT;
    const long long total = (long long)((width + tile_size - 1) / tile_size) * ((height + tile_size - 1) / tile_size);
    return deal_count(tile_deal(world, a, b), (int)total, rank);
}

int pgrt_tile_index_ex(int width, int height, int tile_size, int rank, int world, int a, int b, int j) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || world <= 0 || rank < 0 || rank >= world || j < 0 || a < 0 ||
        b < 0 || a > 64 || b > 64)
        return PGRT_ERR_INVALID_ARGUMENT;
    const int total = ((width + tile_size - 1) / tile_size) * ((height + tile_size - 1) / tile_size);
    const int t = deal_tile(tile_deal(world, a, b), rank, j);
    return t < total ? t : PGRT_ERR_INVALID_ARGUMENT;
}

int pgrt_tile_count(int width, int height, int tile_size, int rank, int world) {
    return pgrt_tile_count_ex(width, height, tile_size, rank, world, 0, 0);
}

int pgrt_tile_index(int width, int height, int tile_size, int rank, int world, int j) {
    return pgrt_tile_index_ex(width, height, tile_size, rank, world, 0, 0, j);
}

int pgrt_tile_share(int world, int* a, int* b) {
    if (world <= 0 || !a || !b) return PGRT_ERR_INVALID_ARGUMENT;
    const TileDeal d = tile_deal(world);
    *a = d.a;
    *b = d.b;
    return PGRT_OK;
}

int pgrt_tile_rect(int width, int height, int tile_size, int t, int rect[4]) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || !rect) return PGRT_ERR_INVALID_ARGUMENT;
    const int tx = (width + tile_size - 1) / tile_size, ty = (height + tile_size - 1) / tile_size;
    if (t < 0 || t >= tx * ty) return PGRT_ERR_INVALID_ARGUMENT;
    rect[0] = (t % tx) * tile_size;
    rect[1] = (t / tx) * tile_size;
    rect[2] = std::min(tile_size, width - rect[0]);
    rect[3] = std::min(tile_size, height - rect[1]);
    return PGRT_OK;
}

int pgrt_unpack_tiles_host(int width, int height, int tile_size, int world, const float* g, float* rgba) {
    return pgrt_unpack_tiles_host_ex(width, height, tile_size, world, 0, 0, g, rgba);
}

int pgrt_unpack_tiles_host_ex(int width, int height, int tile_size, int world, int a, int b, const float* g,
                              float* rgba) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || world <= 0 || !g || !rgba || a < 0 || b < 0 || a > 64 || b > 64)
        return PGRT_ERR_INVALID_ARGUMENT;
    const int tx = (width + tile_size - 1) / tile_size, ty = (height + tile_size - 1) / tile_size;
    const int total = tx * ty;
    const TileDeal d = tile_deal(world, a, b);
    const size_t tile_floats = (size_t)tile_size * tile_size * 4;
    size_t slot = 0;  // rank-major, each rank's tiles in its local order, no padding
    for (int r = 0; r < world; ++r)
        for (int j = 0; j < deal_count(d, total, r); ++j, ++slot) {
            const int t = deal_tile(d, r, j);
            const float* src = g + slot * tile_floats;
            const int x0 = (t % tx) * tile_size, y0 = (t / tx) * tile_size;
            for (int y = 0; y < tile_size && y0 + y < height; ++y)
                for (int x = 0; x < tile_size && x0 + x < width; ++x)
                    std::memcpy(rgba + ((size_t)(y0 + y) * width + (x0 + x)) * 4,
                                src + ((size_t)y * tile_size + x) * 4, 4 * sizeof(float));
        }
    return PGRT_OK;
}

int pgrt_comm_unique_id(char id[128]) {
    if (!id) return PGRT_ERR_INVALID_ARGUMENT;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return PGRT_ERR_RCCL;
    std::memcpy(id, u.internal, 128);
    return PGRT_OK;
}

int pgrt_comm_init(pgrt_ctx* ctx, int world, int rank, const char id[128]) {
    if (!ctx || !id || world <= 0 || world > kMaxRanks || rank < 0 || rank >= world) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(!ctx->group, PGRT_ERR_INVALID_ARGUMENT,
                     "a multi-device context (pgrt_create_devices) has its own communicators");
        drain_frames(ctx);
        if (ctx->comm) {
            (void)ncclCommDestroy(ctx->comm);
            ctx->comm = nullptr;
        }
        ctx->world = world;
        ctx->rank = rank;
        ctx->emulated = false;
        ncclUniqueId u;
        std::memcpy(u.internal, id, 128);
        ncclResult_t r = ncclCommInitRank(&ctx->comm, world, u, rank);
        if (r != ncclSuccess) throw Error(PGRT_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    });
}

int pgrt_comm_info(const pgrt_ctx* ctx, int* nranks, int* rank) {
    if (!ctx || !nranks || !rank) return PGRT_ERR_INVALID_ARGUMENT;
    if (!ctx->comm) {
        *nranks = ctx->world;
        *rank = ctx->rank;
        return PGRT_OK;
    }
    if (ncclCommCount(ctx->comm, nranks) != ncclSuccess || ncclCommUserRank(ctx->comm, rank) != ncclSuccess)
        return PGRT_ERR_RCCL;
    return PGRT_OK;
}

int pgrt_render_distributed_device(pgrt_ctx* ctx, const pgrt_render_params* p, void* rgba_device, pgrt_stats* st) {
    if (!ctx || !p) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        PGRT_REQUIRE(ctx->rank != 0 || rgba_device, PGRT_ERR_INVALID_ARGUMENT, "rank 0 needs an output buffer");
        if (ctx->group) {
            group_render(ctx, p, 1, static_cast<float*>(rgba_device), st);
            return;
        }
        drain_frames(ctx);
        FrameSet* fs = frame_set(ctx, 0);
        // set 0 may last have served pgrt_render_frames_host_async: its host destination belongs
        // to that call (the caller may have freed it), never to this frame
        fs->host_dst = nullptr;
        PGRT_HIP(hipEventRecord(fs->ev_ready, ctx->stream));
        const TileDeal deal = ctx_deal(ctx, ctx->world);
        start_frame(ctx, fs, p, rank_tiles(ctx->cam.width, ctx->cam.height, ctx->rank, deal), nullptr, 1, 0, 0, 0,
                    true, static_cast<float*>(rgba_device), 1, 0, deal);
        fs->pending = false;
        collect_frame(ctx, fs);  // the gather is queued behind the frame (start_frame)
        PGRT_HIP(hipEventRecord(fs->ev_ready, ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
        fs->has_result = true;
        gather_times(fs, &fs->stats);
        fs->stats.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - fs->t0).count();
        if (st) *st = fs->stats;
    });
}

// ---- frames in flight ------------------------------------------------------------------

int pgrt_set_frames_in_flight(pgrt_ctx* ctx, int n) {
    if (!ctx || n < 1 || n > kMaxFramesInFlight) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        drain_frames(ctx);
        ctx->frames_in_flight = n;
        for (pgrt_ctx* m : ctx->members) m->frames_in_flight = n;  // a multi-device context: every rank
    });
}

namespace {
int submit_async(pgrt_ctx* ctx, const pgrt_render_params* p, void* rgba_device, unsigned long long* ticket,
                 bool distributed, int nframes = 1, float* rgba_host = nullptr) {
    if (!ctx || !p || !ticket || (!distributed && !rgba_device && !rgba_host)) return PGRT_ERR_INVALID_ARGUMENT;
    if (nframes < 1 || nframes > kMaxFramesPerCall) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        PGRT_REQUIRE(p->profile == 0, PGRT_ERR_INVALID_ARGUMENT, "profiled frames are synchronous (profile must be 0)");
        PGRT_REQUIRE(!distributed || ctx->rank != 0 || rgba_device, PGRT_ERR_INVALID_ARGUMENT,
                     "rank 0 needs an output buffer");
        if (ctx->group) {  // every rank's tiles, gathered into rgba_device on rank 0
            PGRT_REQUIRE(!rgba_host, PGRT_ERR_INVALID_ARGUMENT,
                         "host-output frames are not available on a multi-device context");
            *ticket = group_submit(ctx, p, nframes, static_cast<float*>(rgba_device));
            return;
        }
        FrameSet* fs = frame_set(ctx, (int)(ctx->next_ticket % (unsigned long long)ctx->frames_in_flight));
        if (fs->pending) finish_through(ctx, fs->ticket);  // the set's previous frame completes first
        fs->host_dst = nullptr;
        // pgrt_config.max_batches_in_flight: bound the sample batches queued across frames in
        // flight (this frame's own count estimated with one slot per frame, as enqueue_frame deals
        // them when frames are in flight)
        if (const int cap = ctx->cfg.max_batches_in_flight; cap > 0) {
            long long nt;
            if (distributed) {
                nt = (long long)rank_tiles(ctx->cam.width, ctx->cam.height, ctx->rank, ctx_deal(ctx, ctx->world)).size();
            } else {
                int x, y, w, h;
                frame_rect(ctx, p, x, y, w, h);
                nt = (long long)((w + kTile - 1) / kTile) * ((h + kTile - 1) / kTile);
            }
            const long long npix = std::max(1ll, nt * nframes) * kTile * kTile;
            const int spp = p->spp_side * p->spp_side;
            const int nsb = (int)std::max(1ll, std::min<long long>(spp, batch_rays(ctx) / npix));
            const int mine = (spp + nsb - 1) / nsb;
            for (;;) {
                int queued = 0;
                unsigned long long oldest = 0;
                for (auto& s : ctx->sets)
                    if (s->pending) {
                        queued += s->batches;
                        if (!oldest || s->ticket < oldest) oldest = s->ticket;
                    }
                if (!oldest || queued + mine <= cap) break;
                finish_through(ctx, oldest);
            }
        }
        if (distributed) {
            const TileDeal deal = ctx_deal(ctx, ctx->world);
            start_frame(ctx, fs, p, rank_tiles(ctx->cam.width, ctx->cam.height, ctx->rank, deal), nullptr, 1, 0, 0,
                        0, true, static_cast<float*>(rgba_device), nframes, 0, deal);
        } else {
            int x, y, w, h;
            frame_rect(ctx, p, x, y, w, h);
            fs->host_dst = rgba_host;
            fs->host_bytes = (size_t)nframes * w * h * 4 * sizeof(float);
            if (rgba_host) {
                fs->host_stage.alloc((size_t)nframes * w * h * 4);
                rgba_device = fs->host_stage.p;
            }
            start_frame(ctx, fs, p, rect_tiles(x, y, w, h), static_cast<float*>(rgba_device), 0, x, y, w, false,
                        nullptr, nframes, (long long)w * h * 4);
        }
        *ticket = fs->ticket;
    });
}
}  // namespace

int pgrt_render_frames_device_async(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes, void* rgba_device,
                                    unsigned long long* ticket) {
    return submit_async(ctx, p, rgba_device, ticket, false, nframes);
}

int pgrt_render_frames_host_async(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes, float* rgba_host,
                                  unsigned long long* ticket) {
    if (!rgba_host) return PGRT_ERR_INVALID_ARGUMENT;
    return submit_async(ctx, p, nullptr, ticket, false, nframes, rgba_host);
}

int pgrt_host_alloc(pgrt_ctx* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
        if (e != hipSuccess) throw Error(PGRT_ERR_OUT_OF_MEMORY, hipGetErrorString(e));
    });
}

int pgrt_host_free(pgrt_ctx* ctx, void* ptr) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] { PGRT_HIP(hipHostFree(ptr)); });
}

int pgrt_render_frames_distributed_device_async(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes,
                                                void* rgba_device, unsigned long long* ticket) {
    return submit_async(ctx, p, rgba_device, ticket, true, nframes);
}

int pgrt_render_device_async(pgrt_ctx* ctx, const pgrt_render_params* p, void* rgba_device,
                             unsigned long long* ticket) {
    return submit_async(ctx, p, rgba_device, ticket, false);
}

int pgrt_render_distributed_device_async(pgrt_ctx* ctx, const pgrt_render_params* p, void* rgba_device,
                                         unsigned long long* ticket) {
    return submit_async(ctx, p, rgba_device, ticket, true);
}

int pgrt_render_wait(pgrt_ctx* ctx, unsigned long long ticket, pgrt_stats* st) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        FrameSet* fs = nullptr;
        for (auto& s : ctx->sets)
            if ((s->pending || s->has_result) && s->ticket == ticket) fs = s.get();
        PGRT_REQUIRE(fs, PGRT_ERR_INVALID_ARGUMENT, "unknown ticket (or its frame set was reused)");
        finish_through(ctx, ticket);
        PGRT_HIP(hipEventSynchronize(fs->ev_ready));
        gather_times(fs, &fs->stats);
        if (st) *st = fs->stats;
    });
}

int pgrt_tune_distribution(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes, void* rgba_device, int calls,
                           int* a_out, int* b_out) {
    if (!ctx || !p || nframes < 1 || nframes > kMaxFramesPerCall || calls < 1 || calls > 64)
        return PGRT_ERR_INVALID_ARGUMENT;
    if (ctx->world <= 1 || (!ctx->comm && !ctx->emulated && !ctx->group)) {  // one rank: nothing to balance
        if (a_out) *a_out = 1;
        if (b_out) *b_out = 1;
        return PGRT_OK;
    }
    // rank 0's share a/8 of another rank's, from half to four times it: below 1 its unpack is the
    // larger cost, above 1 the xGMI ingress of the gather into rank 0 is
    static const int kCand[] = {4, 5, 6, 7, 8, 10, 12, 14, 16, 20, 24, 32};
    const pgrt_config saved = ctx->cfg;
    // every exit restores the caller's configuration unless a share was chosen
    auto fail = [&](int rc) {
        const std::string msg = ctx->err;
        (void)pgrt_set_config(ctx, &saved);
        ctx->err = msg;
        return rc;
    };
    double best = 1e300;
    int best_a = 0;
    for (int a : kCand) {
        pgrt_config c = saved;
        c.rank0_share_a = a;
        c.rank0_share_b = 8;
        int rc = pgrt_set_config(ctx, &c);
        std::vector<unsigned long long> tickets;
        unsigned long long t = 0;
        if (rc == PGRT_OK) rc = pgrt_render_frames_distributed_device_async(ctx, p, nframes, rgba_device, &t);  // warm
        if (rc == PGRT_OK) rc = pgrt_render_wait(ctx, t, nullptr);
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < calls && rc == PGRT_OK; ++k) {
            rc = pgrt_render_frames_distributed_device_async(ctx, p, nframes, rgba_device, &t);
            tickets.push_back(t);
        }
        for (size_t k = 0; k < tickets.size() && rc == PGRT_OK; ++k)
            if (tickets.size() - k <= (size_t)ctx->frames_in_flight) rc = pgrt_render_wait(ctx, tickets[k], nullptr);
        // the slowest rank decides; every rank sees the same maxima, so all pick the same share.
        // A failed rank still joins the reduction with its error flag, so every rank stops here
        // together instead of waiting in the next candidate's collectives
        double v2[2] = {std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                        rc == PGRT_OK ? 0.0 : 1.0};
        const int rrc = guarded(ctx, [&] {
            // emulation: this rank's time alone; a multi-device context timed every rank itself
            if (!ctx->comm || ctx->group) return;
            DevBuf<double> v;
            v.alloc(2);
            PGRT_HIP(hipMemcpyAsync(v.p, v2, sizeof(v2), hipMemcpyHostToDevice, ctx->stream));
            const ncclResult_t r = ncclAllReduce(v.p, v.p, 2, ncclFloat64, ncclMax, ctx->comm, ctx->stream);
            if (r != ncclSuccess) throw Error(PGRT_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
            PGRT_HIP(hipMemcpyAsync(v2, v.p, sizeof(v2), hipMemcpyDeviceToHost, ctx->stream));
            PGRT_HIP(hipStreamSynchronize(ctx->stream));
        });
        if (rc != PGRT_OK) return fail(rc);
        if (rrc != PGRT_OK) return fail(rrc);
        if (v2[1] != 0.0) {
            ctx->err = "pgrt_tune_distribution: another rank failed";
            return fail(PGRT_ERR_RCCL);
        }
        if (v2[0] < best) {
            best = v2[0];
            best_a = a;
        }
    }
    pgrt_config c = saved;
    c.rank0_share_a = best_a;
    c.rank0_share_b = 8;
    const int rc = pgrt_set_config(ctx, &c);
    if (rc != PGRT_OK) return fail(rc);
    if (a_out) *a_out = best_a;
    if (b_out) *b_out = 8;
    return PGRT_OK;
}

int pgrt_unpack_tiles_device(pgrt_ctx* ctx, int width, int height, int world, int a, int b, const void* tiles_device,
                             void* rgba_device) {
    if (!ctx || width <= 0 || height <= 0 || world <= 0 || world > kMaxRanks || a < 0 || b < 0 || a > 64 || b > 64 ||
        !tiles_device || !rgba_device)
        return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        const TileDeal d = tile_deal(world, a, b);
        UnpackSrc u = unpack_layout(d, width, height);
        const float* g = static_cast<const float*>(tiles_device);
        for (int r = 0; r < world; ++r) u.src[r] = g + (size_t)u.prefix[r] * kTile * kTile * 4;
        launch_unpack_tiles(u, static_cast<float*>(rgba_device), width, height, d, 4, ctx->stream, 0, 1);
        PGRT_HIP(hipGetLastError());
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int pgrt_render_tiles_device(pgrt_ctx* ctx, const pgrt_render_params* p, int rank, int world, void* tiles_device,
                             pgrt_stats* st) {
    if (!ctx || !p || !tiles_device || world <= 0 || rank < 0 || rank >= world) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        auto t0 = std::chrono::steady_clock::now();
        render_tiles(ctx, p, rank_tiles(ctx->cam.width, ctx->cam.height, rank, ctx_deal(ctx, world)),
                     static_cast<float*>(tiles_device), 1, 0, 0, 0, st);
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
        if (st) st->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    });
}

int pgrt_render_distributed(pgrt_ctx* ctx, const pgrt_render_params* p, float* rgba_host, pgrt_stats* st) {
    if (!ctx || !p) return PGRT_ERR_INVALID_ARGUMENT;
    const int W = ctx->cam.width, H = ctx->cam.height;
    int rc = guarded(ctx, [&] {
        PGRT_REQUIRE(ctx->has_cam, PGRT_ERR_NO_CAMERA, "pgrt_set_camera has not been called");
        if (ctx->rank == 0) ctx->fb_dev.alloc((size_t)W * H * 4);
    });
    if (rc != PGRT_OK) return rc;
    rc = pgrt_render_distributed_device(ctx, p, ctx->rank == 0 ? ctx->fb_dev.p : nullptr, st);
    if (rc != PGRT_OK || ctx->rank != 0 || !rgba_host) return rc;
    return pgrt_copy_to_host(ctx, rgba_host, ctx->fb_dev.p, (size_t)W * H * 4 * sizeof(float));
}

int pgrt_timeline_enable(pgrt_ctx* ctx, int on) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        drain_frames(ctx);  // pending frames were enqueued with the old choice
        ctx->timeline_on = on != 0;
    });
}

int pgrt_timeline_read(pgrt_ctx* ctx, pgrt_timeline_rec* out, int max, int* n) {
    if (!ctx || !n || max < 0 || (max > 0 && !out)) return PGRT_ERR_INVALID_ARGUMENT;
    const int k = (int)std::min<size_t>((size_t)max, ctx->timeline.size());
    std::copy(ctx->timeline.begin(), ctx->timeline.begin() + k, out);
    ctx->timeline.erase(ctx->timeline.begin(), ctx->timeline.begin() + k);
    *n = k;
    return PGRT_OK;
}

int pgrt_frame_diag(const pgrt_ctx* ctx, pgrt_level_diag* out, int max_levels) {
    if (!ctx || !out || max_levels <= 0) return PGRT_ERR_INVALID_ARGUMENT;
    const int n = std::min(max_levels, kMaxLevels);
    std::memset(out, 0, sizeof(pgrt_level_diag) * n);
    for (const FrameCounters& h : ctx->last_fc)
        for (int L = 0; L < n; ++L) {
            pgrt_level_diag& d = out[L];
            d.rays += (uint64_t)fc_count(h, L);
            d.shadow_rays += (uint64_t)fc_shadow(h, L);
            d.visits += h.trav[L][0] + h.trav[L][14];
            d.wide_visits += h.trav[L][14];
            d.tests += h.trav[L][1];
            d.max_visits = std::max<uint64_t>(d.max_visits, h.trav[L][2]);
            d.max_tests = std::max<uint64_t>(d.max_tests, h.trav[L][3]);
            d.max_wave_iterations = std::max<uint64_t>(d.max_wave_iterations, h.trav[L][4]);
            d.max_ray_ticks = std::max<uint64_t>(d.max_ray_ticks, h.trav[L][5]);
            d.stack_spills += h.trav[L][6];
            d.max_stack = std::max<uint64_t>(d.max_stack, h.trav[L][7]);
            for (int k = 0; k < 6; ++k)
                d.longest_ray[k] = std::max<uint64_t>(d.longest_ray[k], h.trav[L][8 + k] & 0xffffffull);
            d.ms_trace = ctx->level_ms[L][0];
            d.packet_steps_hit += h.pkt[L][0];
            d.packet_steps_live += h.pkt[L][1];
            d.ms_shade = ctx->level_ms[L][1];
            d.shadow_visits += h.trav[kMaxLevels + L][0];
            d.shadow_tests += h.trav[kMaxLevels + L][1];
            d.shadow_max_visits = std::max<uint64_t>(d.shadow_max_visits, h.trav[kMaxLevels + L][2]);
            d.shadow_max_tests = std::max<uint64_t>(d.shadow_max_tests, h.trav[kMaxLevels + L][3]);
        }
    return n;
}

// test hook: device evaluation of the shared math (sqrt, div, powf, expf, atan2f, asinf, rsqrt, pow)
int pgrt_selftest_math(pgrt_ctx* ctx, const float* in_pairs, int n, float* out8) {
    if (!ctx || n < 0 || (n > 0 && (!in_pairs || !out8))) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        if (n == 0) return;
        DevBuf<float> a, b;
        a.alloc((size_t)2 * n);
        b.alloc((size_t)8 * n);
        PGRT_HIP(hipMemcpyAsync(a.p, in_pairs, sizeof(float) * 2 * n, hipMemcpyHostToDevice, ctx->stream));
        launch_selftest_math(a.p, n, b.p, ctx->stream);
        PGRT_HIP(hipGetLastError());
        PGRT_HIP(hipMemcpyAsync(out8, b.p, sizeof(float) * 8 * n, hipMemcpyDeviceToHost, ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
    });
}

// test hook: the kernels' sRGB expand / compress against their exact form over a float range
int pgrt_selftest_srgb(pgrt_ctx* ctx, uint32_t first_bits, uint32_t count, uint64_t* mismatches) {
    if (!ctx || !mismatches) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        DevBuf<unsigned long long> m;
        m.alloc(2);
        PGRT_HIP(hipMemsetAsync(m.p, 0, 2 * sizeof(unsigned long long), ctx->stream));
        launch_selftest_srgb(first_bits, count, m.p, ctx->stream);
        PGRT_HIP(hipGetLastError());
        unsigned long long h[2] = {0, 0};
        PGRT_HIP(hipMemcpyAsync(h, m.p, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
        PGRT_HIP(hipStreamSynchronize(ctx->stream));
        mismatches[0] = h[0];
        mismatches[1] = h[1];
    });
}

}  // extern "C"
