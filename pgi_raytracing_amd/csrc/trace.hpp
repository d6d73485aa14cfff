// trace.hpp -- launchers of the hand-written gfx950 kernels (host-callable).
#pragma once

#include "common.hpp"

namespace pgrt {

// traversal stack: kLdsStack entries per lane in LDS (16 x 4 B x 256 lanes = 16 KB per block,
// so LDS does not cap occupancy below the VGPR limit), deeper entries in a per-thread global
// region of kGlobalStack entries
constexpr int kLdsStack = 16;
constexpr int kGlobalStack = 112;
constexpr int kTile = 64;         // image tile side (multi-GPU unit, level-0 ray order)
constexpr int kMaxLevels = 16;    // max_level + 1 <= kMaxLevels

// Per-frame device counters (zeroed by one hipMemsetAsync per batch).
struct FrameCounters {
    // queue allocation: shade(L) reserves its children (level L+1 rays) and its shadow rays with
    // ONE 64-bit atomic per wave on alloc[L] = shadow rays of L << 32 | rays of level L+1 (the low
    // word never carries: counts stay below 2^31); level 0's count is written by raygen.  Read
    // them through fc_count / fc_shadow.
    int count0;
    int overflow;                        // set when an emit exceeded a queue capacity
    int pad0[2];
    unsigned long long alloc[kMaxLevels];
    // statistics only (fire-and-forget atomics), on cache lines of their own so they never
    // serialise with the allocation atomics
    alignas(128) int refract[kMaxLevels];  // refraction rays among the rays of level L
    // profile == 2: per closest-hit launch {sum node visits, sum triangle tests, max visits of
    // one ray, max tests of one ray}; [0, kMaxLevels) level queues, [kMaxLevels, 2k) shadows
    alignas(128) unsigned long long trav[2 * kMaxLevels][16];  // visits, tests, max visits, max tests, max wave iterations
    // packet traversal utilisation per level (sampled blocks): {lane-steps whose ray hit a child
    // box, live lane-steps}; filled only by levels traced as packets
    alignas(128) unsigned long long pkt[kMaxLevels][2];
    // profile == 2: per level, shaded rays that hit a triangle and, of those, the ones whose
    // Phong branch sampled a texture (the whole-frame roofline's attribute / texel bytes)
    alignas(128) unsigned long long shade[kMaxLevels][2];
    // packet launches with a step budget (pgrt_config.packet_budget): rays of the waves that ran
    // out of steps, finished by the 8-lanes-per-ray kernel (count; the list is FrameSlot::q_defer)
    alignas(128) int defer[kMaxLevels];
    int probe_defer;  // the AUTO probe's deferral count (its side launch; never read)
};

__host__ __device__ inline int fc_count(const FrameCounters& f, int L) {
    return L == 0 ? f.count0 : (int)(unsigned)(f.alloc[L - 1] & 0xffffffffull);
}
__host__ __device__ inline int fc_shadow(const FrameCounters& f, int L) { return (int)(unsigned)(f.alloc[L] >> 32); }
// device address of level L's ray count (a trace launch reads it); shadow counts are the high
// words of alloc[0..levels), stride 2 ints (fc_shadow_counts)
inline int* fc_count_ptr(FrameCounters* f, int L) {
    return L == 0 ? &f->count0 : reinterpret_cast<int*>(&f->alloc[L - 1]);
}
inline int* fc_shadow_counts(FrameCounters* f) { return reinterpret_cast<int*>(&f->alloc[0]) + 1; }

constexpr int kXcds = 8;  // MI355X: workgroups are dispatched round-robin over 8 XCDs

struct FrameParams {
    int spp_side;
    int max_level;
    int dof;
    float focal, aperture, gamma;
    int jitter;
    unsigned seed, frame;
    int s0, nsb;   // first sample and samples in this batch
    int ntiles;
    // multi-frame calls: the caller's tile list is nframes copies of one frame's tiles
    // (frame-major); a slot's tile q is the caller's tile q * slots + slot, its frame that index
    // / frame_tiles (frame_tiles 0: one frame).  Frame f jitters with frame index frame + f and
    // writes a framebuffer at out + f * frame_stride floats (tile-compact outputs are frame-major).
    int slots, slot, frame_tiles, frame_out_tiles;  // frame_out_tiles: tiles per frame in a tile-compact output
    long long frame_stride;
    int count;  // profile == 2: the shade kernels count hits / textured hits (FrameCounters::shade)
    // get_pixel's per-frame constants (host IEEE float divisions = the device's correctly rounded
    // ones): 1 / S and the sub-pixel jitter interval [-0.5 / S, 0.5 / S] (raytracer.cpp:407-413)
    float inv_s, jit_a, jit_b;
    // synchronous frames: the level-0 shade sets tile_deep[q] = 1 for the slot's tile q when a
    // primary ray there hit a dielectric (reflection / refraction children) -- the next frame's
    // tile deal (context.cpp deal_tiles); NULL: not recorded
    int* tile_deep;
};

// A tile record is (x, y, width | frame << 8, height): the frame of a multi-frame call the tile
// belongs to rides in the record (set by start_frame), so no ray divides by the call's tile count
constexpr int kTileFrameShift = 8;
__host__ __device__ inline int tile_width(const int4& tr) { return tr.z & ((1 << kTileFrameShift) - 1); }
__host__ __device__ inline int frame_of_tile(const int4& tr) { return tr.z >> kTileFrameShift; }

// level-L queue view
struct Queue {
    float4* ro;      // org.xyz, tnear
    float4* rd;      // dir.xyz, tfar
    float* time;     // medium IOR (RTCRay::time as used by the reference)
    float4* hit;     // t, u, v, prim bits
    int cap;
};

// direction octant of a ray: the sign bits the packet traversal specialises its node loop on
// (bit 0: x < 0, bit 1: y < 0, bit 2: z < 0; -0 counts as negative, as rcp(-0) < 0)
__device__ inline unsigned dir_octant(float x, float y, float z) {
    return (__float_as_uint(x) >> 31) | ((__float_as_uint(y) >> 31) << 1) | ((__float_as_uint(z) >> 31) << 2);
}

// Where a batch's finished pixels go (k_finish; the level-0 packet traversal for primary-ray
// misses of a 1-spp frame).  mode 0: framebuffer (rect origin ox,oy, row pitch in pixels);
// 1: tile-compact RGBA; 2: tile-compact RGB (the multi-GPU gather format).  The launch's tiles
// are tiles j, j + K, ... of the caller's list (pipeline slot j of K).
struct FrameOut {
    float* out;
    int mode, ox, oy, pitch, K, j;
};

// Level 0 of a 1-spp batch traced as packets (PrimaryGen): a pixel whose primary ray misses has
// one colour, the environment texel (raytracer.cpp:390-393), so get_pixel's sum and gamma
// (:422-435) follow in the level-0 shade, which writes it to fo at once -- no node record, no
// finish.  hit: per 64-ray wave, the lanes whose ray hit (the traversal stores no hit record for
// a miss); pending: per wave, the lanes the finish still has to complete (set by the shade).
struct L0Final {
    unsigned long long* hit;
    unsigned long long* pending;
    FrameOut fo;
    const int4* tiles;
    // one light, compact shadow queue (ShadowFinal): an opaque pixel with a shadow ray is completed
    // by the shadow trace (its pixel travels in the ray's Phong term), not by the finish; an opaque
    // pixel without one has its final colour already and is written here like a miss
    int shadow_final = 0;
};

// Level 0 of such a batch (L0Final.shadow_final): the shadow queue's first fc_shadow(0) rays are
// the level-0 pixels' only shadow rays, contrib.w = the pixel's slot index.  The shadow trace
// completes each of those pixels -- opaque_color (lit: the Phong term, else 0) and get_pixel's
// sum and gamma (raytracer.cpp:163-173, 344-386, 422-435) -- so k_finish_pending is left with the
// dielectric pixels.  contrib NULL: off.
// Levels 1 .. levels-1 likewise (colors[L] non-NULL): an opaque node's only shadow ray carries its
// node index, and the shadow trace writes the node's colour (opaque_color), so k_combine skips it.
struct ShadowFinal {
    const float4* contrib = nullptr;
    const int* n0 = nullptr;  // &fc_shadow(0) (FrameCounters::alloc's high word of level 0), stride 2
    FrameParams fp{};
    const int4* tiles = nullptr;
    FrameOut fo{};
    int levels = 0;                       // levels whose shadow rays are in the queue (count terms)
    float4* colors[kMaxLevels] = {};      // colors[L]: level L's node colours (L >= 1), NULL: off
};

struct LevelNodes {  // per-level node records kept until the combine pass
    float4* color;
    int4* link;      // dielectric: (refl child, refr child or -1, -, -); opaque: (-1,-1,shadow base, n)
    float4* att;     // dielectric: (att.r, att.g, att.b, R)
};

struct ShadowQueue {  // one per batch: the shadow rays of every level, level-major
    float4* ro;       // NULL in the compact form (one light: every shadow ray starts at it)
    float4* rd;
    float4* hit;      // closest hits (full form); NULL in the compact form
    float4* contrib;  // (blue, green, red, owner) Phong term of the owning node for this light; w = the
                      // owner node as int bits when the shadow trace completes it (ShadowFinal), else unused
    int cap;
    // compact form (one light, binary BVH): the shadow trace writes is_illuminated's verdict
    // (raytracer.cpp:163-173: no hit, or a hit on a dielectric) as one byte per ray instead of a
    // 16-B hit record, and reads no origin (LightSource::GenerateRay: org = the light)
    unsigned char* lit;
};

// One closest-hit launch over a ray queue (ro/rd in, hits out).  Ray count: the sum of
// count_dev[0], count_dev[2], ... (count_terms words, stride 2: FrameCounters::alloc) clamped to
// max_count when count_dev is set, else count_host.  expect sizes the grid only (counts live on
// the device; last frame's count avoids dispatching empty workgroups).  Kernel choice: gen
// (level 0: rays generated in registers) or packets -> wave packets over the binary BVH; queues
// of <= group_max rays (allow_group) -> 8 / 4 lanes per ray over the 8-wide BVH; else one lane
// per ray.  count: profile == 2 traversal counters into counters[16].
struct PrimaryGen;  // camera_ops.hpp
struct TraceLaunch {
    int level = -1;  // queue level (timeline records), -1: none / the shadow queue
    const float4* ro = nullptr;
    const float4* rd = nullptr;
    float4* hits = nullptr;
    const int* count_dev = nullptr;
    int count_terms = 1;
    int count_host = 0;
    int max_count = 0;
    int expect = 0;
    int* gstack = nullptr;  // per-thread global stack region (one-lane kernels)
    int gstack_threads = 0;
    unsigned long long* counters = nullptr;
    bool count = false;
    bool allow_group = true;
    bool packets = false;
    const PrimaryGen* gen = nullptr;
    unsigned long long* pkt_util = nullptr;  // packet launches: sampled utilisation sums (FrameCounters::pkt)
    // shadow queues in the compact form (one-lane kernel): ro == NULL -> every ray starts at
    // const_org (xyz, tnear in w); lit != NULL -> write is_illuminated's byte, not the hit
    float4 const_org = make_float4(0, 0, 0, 0);
    unsigned char* lit = nullptr;
    // bounce-level packets (packets && !gen): a wave still traversing after `budget` node /
    // triangle steps stores its rays' closest hits so far and appends the rays to defer_list
    // (count in *defer_count); a second launch finishes them 8 lanes per ray over the 8-wide BVH,
    // starting from those hits.  budget 0: no budget.  defer_expect sizes its grid.
    int budget = 0;
    int* defer_list = nullptr;
    int* defer_count = nullptr;
    int defer_expect = 0;
    bool resume = true;  // false: the deferred rays are not finished (a side launch that only samples)
    ShadowFinal sfin;    // the compact shadow queue of a 1-spp batch: level-0 pixels completed here
};
// the packet traversal needs the binary layout and a tree that fits its wave-uniform stack
bool trace_packets_available(const SceneView& s);
// returns false when nothing was launched (max_count <= 0)
bool launch_trace(const SceneView& s, const TraceLaunch& t, hipStream_t stream);
// events the next launch_trace records at its kernel's start / end (nullptr: none)
void set_trace_events(hipEvent_t start, hipEvent_t stop);
int trace_block_size();
// any-hit query (rtcOccluded1 semantics): occluded[i] = 1 when some triangle is hit in (tnear, tfar]
void launch_occluded(const SceneView& s, const float4* ro, const float4* rd, int n, int* occluded,
                     hipStream_t stream);

// `expect` sizes the grid of a grid-stride kernel (counts live on the device; any value is
// correct, a good guess -- last frame's count -- avoids dispatching empty workgroups)
void launch_raygen(const CameraView& cam, const FrameParams& fp, const int4* tiles, Queue q, int n0,
                   FrameCounters* fc, hipStream_t stream);
// level 0 of a pinhole frame traced as packets: the queue holds only directions (rd); every
// valid ray starts at the camera (x, y, z) with tnear 0.001, in air
struct PinholeOrigin {
    float x, y, z;
    int on;
};
// l0f.hit != NULL: level 0 of a 1-spp batch (L0Final)
void launch_shade(const SceneView& s, const FrameParams& fp, int level, Queue q, Queue next, LevelNodes nodes,
                  ShadowQueue sq, FrameCounters* fc, int max_count, hipStream_t stream, int expect,
                  const PinholeOrigin& l0, const L0Final& l0f);
// level L's final colours from its shadow hits and level L+1's colours (child)
void launch_combine(const SceneView& s, int level, LevelNodes nodes, const float4* child, ShadowQueue sq,
                    const FrameCounters* fc, int max_count, hipStream_t stream, int expect = 0);
// level-0 combine + sample accumulation (+ gamma and the output write on the last batch, fo).
// resolved: level 0's final colours were written by launch_combine(level 0) (several samples
// per pixel).  l0f.pending != NULL (1 spp, L0Final): only the pixels whose bit is set there are
// finished (the others were written by the level-0 shade).
void launch_finish(const SceneView& s, const FrameParams& fp, const int4* tiles, LevelNodes l0, const float4* child,
                   ShadowQueue sq, float4* accum, const FrameOut& fo, int npix, bool first, bool last,
                   bool resolved, const unsigned long long* pending, hipStream_t stream);
// frame sink: sum += frame (count-th frame; count == 1 resets), mean = sum / count
void launch_accumulate_frame(const float* frame, float* sum, float* mean, long long pixels, int count,
                             hipStream_t stream);
// The deep Whitted levels as one launch (subtree.hip): every ray of level `level` (queue q, count
// fc_count(level)) evaluates its whole ray tree depth first -- reflection, refraction and shadow
// rays traced by 8 (4) lanes per ray over the 8-wide BVH -- and writes its final colour as a
// level-`level` node record (k_combine of level - 1 reads it); the per-level statistics of the
// deeper levels are counted as k_shade counts them.  expect sizes the grid; count: profile == 2
// traversal / shading counters.
constexpr int kSubtreeGroup8Max = 150000;  // 4 lanes per ray above this many rays (as kGroup8Max)
bool subtree_available(const SceneView& s);
void launch_subtree(const SceneView& s, const FrameParams& fp, int level, Queue q, LevelNodes nodes,
                    FrameCounters* fc, int max_count, int expect, bool count, hipStream_t stream);
// copy `n` FrameCounters to pinned host memory and zero them on the device
// also copies the slot's per-tile deep flags (FrameParams::tile_deep, ndeep ints) to deep_host and
// zeroes them on the device (deep_dev NULL: none)
// host-output frames: a pipeline slot's finished tiles (ntiles records, frame index in each) from
// the device framebuffer src to the same place in the page-locked host framebuffer dst_host
// (device-visible address); framebuffer origin ox, oy, pitch in pixels, frame_stride in floats
void launch_export_tiles(const int4* tiles, int ntiles, const float* src, float* dst_host, int ox, int oy, int pitch,
                         long long frame_stride, hipStream_t stream);
// the first `bytes` of a device framebuffer into page-locked host memory (device-visible address)
void launch_blit_host(const float* src, float* dst_host, size_t bytes, hipStream_t stream);
void launch_export_counters(FrameCounters* dev, FrameCounters* host, int n, int* deep_dev, int* deep_host, int ndeep,
                            hipStream_t stream);
// Distributed frames: rank r's tile-compact buffer (frame-major, count[r] tiles per frame in its
// local deal order); prefix = exclusive prefix of the counts (prefix[world] = all tiles)
constexpr int kMaxRanks = 16;
struct UnpackSrc {
    const float* src[kMaxRanks];
    int count[kMaxRanks];
    int prefix[kMaxRanks + 1];
};
struct TileDeal;  // tiles.hpp
// unpack frames frame0 .. frame0 + nframes - 1 of every rank's tiles into rgba (W*H*4 floats per
// frame); channels 4 (RGBA tiles) or 3 (RGB tiles, alpha 1: the gather format)
void launch_unpack_tiles(const UnpackSrc& u, float* rgba, int width, int height, const TileDeal& deal, int channels,
                         hipStream_t stream, int frame0, int nframes);
// Distributed frames without a control collective: a rank's send carries, after its tiles, a tail
// of kGatherTail floats whose first word is its queue-overflow flag (the OR of every slot's and
// batch's FrameCounters::overflow, read from the exported counters); rank 0 copies every peer's
// flag into host memory.  fcs[j]: slot j's exported counters (host-mapped), n[j] batches.
constexpr int kGatherTail = 4;
struct FlagSrc {
    const FrameCounters* fc[4];
    int n[4];
    int K;
    int poison;    // this rank gave up re-rendering the frame: its tiles are garbage (flag 2)
    unsigned seq;  // the rank's distributed-frame sequence number (tail word 1): rank 0 checks it
};
// tail words: [0] 0 = complete, 1 = queues overflowed (a re-send follows), 2 = gave up; [1] seq
void launch_overflow_flag(const FlagSrc& f, int* out, hipStream_t stream);
// flags[r] = the flag word after rank r's `floats` floats of tiles at u.src[r] (r = 1 .. world-1)
// flags[r] / flags[kMaxRanks + r] = tail words 0 / 1 of rank r's send (0 for ranks not received)
void launch_peer_flags(const UnpackSrc& u, int world, size_t floats_per_tile_count, int* flags, hipStream_t stream);

// scene / BVH build
constexpr int kBuilderLbvh = PGRT_BVH_LBVH;  // Karras 2012 over 63-bit Morton codes
constexpr int kBuilderPloc = PGRT_BVH_PLOC;  // PLOC clustering over the same Morton order + SAH collapse
constexpr int kDefaultSlots = 2;           // pipeline slots of a synchronous frame (r1 A/B: 2 > 1, 3)
constexpr int kDefaultGroupMax = 400000;   // pgrt_config.group_max default: queues up to this many rays use
                                           // the 8-lanes-per-ray kernel (r1 A/B: tail levels -45 %)
constexpr int kDefaultGroupMaxInFlight = 100000;  // with frames in flight the concurrent frames hide
                                                  // the latency floors: level 2 (~150k rays) runs
                                                  // faster one lane per ray (r1 scan: 0.392 -> 0.366)
// pgrt_config.packet_budget default: node / triangle steps a bounce-level packet wave takes before
// its rays go to the 8-lanes-per-ray kernel (calibrated on C2)
constexpr int kDefaultPacketBudget = 256;
// batches below kSmallPacketBatch level-0 rays (one 1080p frame: 2.1M) take the shorter budget
// on their bounce levels (context.cpp packet_budget)
constexpr int kSmallPacketBatch = 1 << 22;
constexpr int kSmallBatchPacketBudget = 64;
// one-frame batches: levels >= this as whole ray trees in one launch (pgrt_config.subtree_level);
// synchronous frames (one frame in flight) from level 2 (r5za: 0.556 -> 0.530 ms), one-frame calls
// in flight from level 3 (from level 2 their throughput drops: 0.255 -> 0.290 ms/frame)
constexpr int kSubtreeLevelSmall = 3;
constexpr int kSubtreeLevelSync = 2;
// "big" scenes (BVH + triangles far beyond the L2, fetches served by the MALL / HBM): the
// level-0 packet kernel is built for 8 waves (trace.hip), level 0 of calls in flight is ordered
// (context.cpp call_ordered)
constexpr int kPacketBigScene = 262144;
struct BuildOut {
    int builder;   // in: kBuilder*
    int leaf_max;  // in: triangles per binary leaf (<= kLeafMaxTris)
    int root;
    int num_nodes;
    int max_depth;
    int iterations;  // PLOC merge iterations
    int refs;        // leaf entries (triangle references; == triangles without splitting)
};
void build_ploc(const float* pos_dev, const float4* ref_lo, const float4* ref_hi, const int* order, int nref,
                float4* tri_out, BvhNode* nodes_out, BuildOut* out, int* iterations, hipStream_t stream);
// PLOC over triangle references (split.hip): beta > 0 adds up to beta * n split references
// (early split clipping); sizes tri (3 float4 per reference) and nodes; returns the count
int build_ploc_refs(const float* pos_dev, int ntri, float beta, float pad, float extent, DevBuf<float4>& tri,
                    DevBuf<BvhNode>& nodes, BuildOut* out, hipStream_t stream);
void build_lbvh(const float* pos_dev, int ntri, float4* tri_out, BvhNode* nodes_out, int* scratch_int,
                void* sort_tmp, size_t sort_tmp_bytes, float pad, BuildOut* out, hipStream_t stream);
// collapse the binary BVH (root: node index or leaf code; root box used for a leaf root) into
// the 8-wide quantized layout; tri_out receives the triangles in wide-leaf order
// Ng = e2 x e1 per BVH reference (SceneView::tri_ng), same float operations as tri_test
void compute_tri_normals(const float4* tri, int m, float4* ng, hipStream_t stream);
void build_bvh8(const BvhNode* bin, const float4* tri_in, int root, int n, float4 root_lo, float4 root_hi,
                Bvh8Node* out, float4* tri_out, int* num_nodes, int* depth, hipStream_t stream);
size_t lbvh_sort_temp_bytes(int ntri);
size_t lbvh_scratch_ints(int ntri);
void launch_pack_attributes(const float* nrm, const float* uv, const int* mat, int ntri, float* attr,
                            hipStream_t stream);

// math self-test hook (tests/test_gpu_*): evaluates the shared math on the device
void launch_selftest_math(const float* in, int n, float* out, hipStream_t stream);
void launch_selftest_srgb(uint32_t first_bits, uint32_t count, unsigned long long* mismatches, hipStream_t stream);

}  // namespace pgrt
