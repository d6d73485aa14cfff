// frame.cpp -- frame scheduling: pipeline slots and their buffers, the tile deal, the per-level
// launch sequence of a frame (enqueue_frame: Raytracer::trace's recursion, APP/raytracer.cpp:237-394,
// as one ray queue per level), the frame counters, the queue-overflow re-render and the frame
// statistics; the synchronous and asynchronous frame entry points build on start_frame /
// finish_through.
#include "context.hpp"

using namespace pgrt;

// ShadowFinal (A/B switch, compile time): 1 = level-0 opaque pixels of 1-spp batches with one light
// are completed by the shadow trace
#ifndef PGRT_SHADOW_FINAL
#define PGRT_SHADOW_FINAL 1
#endif
// ... and at every level below the subtree launch (the opaque nodes' colours; A/B switch)
#ifndef PGRT_SHADOW_FINAL_ALL
#define PGRT_SHADOW_FINAL_ALL 1
#endif

namespace pgrt {

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

// The tiles of each pipeline slot.  Round-robin (slot j gets tiles j, j + K, ...; tile-compact and
// distributed outputs rely on it: store_pixel's position in the caller's tile list; a multi-frame
// call's tile records carry their frame index, frame_of_tile).
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
// Default: one-frame batches of scenes up to kPacketBigScene triangles -- synchronous frames from
// level kSubtreeLevelSync, one-frame calls in flight from kSubtreeLevelSmall (the synchronous
// frame's deep levels are a few ten thousand rays whose per-level launches each last as long as
// their slowest ray; r4l timeline 0.583-0.597 -> 0.563 ms from level 3, r5za 0.556 -> 0.530 ms
// from level 2; calls in flight lose throughput from level 2: 0.255 -> 0.290 ms/frame), one
// launch per level otherwise (the subtree launch's 8 lanes per ray cost multi-frame calls
// throughput: r4h driver line 0.179 -> 0.209 ms/frame).
int subtree_first(const pgrt_ctx* ctx, const SceneView& view, const pgrt_render_params* p, bool small_batch) {
    const int k = ctx->cfg.subtree_level;
    if (k < 0 || p->mode != PGRT_MODE_WHITTED || !subtree_available(view)) return -1;
    if (k > 0) return k <= p->max_level ? k : -1;
    const int first = ctx->frames_in_flight > 1 ? kSubtreeLevelSmall : kSubtreeLevelSync;
    return small_batch && view.ntri <= kPacketBigScene && first <= p->max_level ? first : -1;
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
    // one probe per re-probe period: the launch sits on the call's level chain (~0.1 ms at C2's level
    // 3, as long as its slowest packet wave), and every call submitted before the next collect would
    // otherwise probe as well (8 calls in flight: up to 8 probes per period)
    ctx->probe_level = -1;
}

// How a host-output frame's pixels reach host memory (pgrt_config.host_export): per slot by the
// export kernel (page-locked destinations only), right after the slot's finish -- so the bulk
// slot's pixels cross PCIe while the deep-tile slot of a synchronous frame still renders -- or by
// one DMA copy after every slot.  r5d / r5e A/B (same box, profiles/r5): one synchronous C2 frame
// into page-locked memory 1.69 ms with one copy after the frame, 1.02 with per-slot export kernels
// of 32 workgroups (1.14 with 256: the kernel's PCIe stores stall the memory pipelines of CUs the
// deep-tile slot also runs on), 5.2 with per-slot DMA copies of the slot's tile runs (2D copies);
// calls in flight 0.61-0.65 ms/frame with one DMA copy per call, 0.76-0.83 with export kernels
// (their stores slow the other calls' rendering).  But a process's SDMA rate is not fixed: the
// same copy runs at 27 or 54 GB/s (r5k / r5l / r5n probes: typically the first process on a box),
// where the blit kernel stays at 53-54.  In-process A/B on a fast-SDMA box (r5m, 8 frames x 4
// calls): DMA 0.63-0.76 ms/frame, half kernel + half DMA concurrently (split) 0.656-0.66, export
// kernels 0.67-0.69; on slow-SDMA boxes the bench line read DMA 0.93-0.96 (r5fin) and split 0.84
// (r5fin2).  So every page-locked destination takes the export kernels by default -- the one form
// whose rate does not depend on the box -- and split / DMA stay selectable.
enum { kHostNone = 0, kHostKernel = 1, kHostOnce = 2, kHostSplit = 3 };
int host_export_mode(const pgrt_ctx* ctx, const FrameSet* fs, int K) {
    if (!fs->host_dst || K == 0) return kHostNone;
    const int c = ctx->cfg.host_export;
    if (c == PGRT_HOST_EXPORT_COPY || !fs->host_map) return kHostOnce;
    if (c == PGRT_HOST_EXPORT_KERNEL) return kHostKernel;
    if (c == PGRT_HOST_EXPORT_SPLIT) return kHostSplit;
    return kHostKernel;
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
    const int hx = host_export_mode(ctx, fs, K);
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
            // one light over the binary BVH: the level-0 opaque pixels are completed by the shadow
            // trace (ShadowFinal), the finish keeps the dielectric ones
            const bool shadow_final = PGRT_SHADOW_FINAL && l0final && compact_shadow && p->max_level > 0;
            // ... and the opaque nodes of the deeper levels get their colour there (k_combine skips them)
            const bool shadow_final_all = shadow_final && PGRT_SHADOW_FINAL_ALL;
            const L0Final l0f{l0final ? sl->l0_hit.p : nullptr, l0final ? sl->l0_pending.p : nullptr, fo,
                              sl->tiles.p, shadow_final ? 1 : 0};
            const PrimaryGen gen{ctx->cam, fp, sl->tiles.p, dir_only ? nullptr : q[0].ro, q[0].rd,
                                 dir_only ? nullptr : q[0].time, &fcd->count0, l0f.hit};
            int id = ctx->timer.begin(s, CAT_RAYGEN);
            if (!fuse) launch_raygen(ctx->cam, fp, sl->tiles.p, q[0], n0, fcd, s);
            debug_sync(s, "raygen", 0, bi);
            ctx->timer.end(s, id);
            // levels >= sub: whole ray trees in one launch (no queues, shades or combines below it)
            const int sub = subtree_first(ctx, view, p, n0 < kSmallPacketBatch);
            sl->sub_first = sub;
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
                             L == 0 ? l0f : L0Final{nullptr, nullptr, fo, nullptr, shadow_final_all ? 1 : 0});
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
                if (shadow_final) {
                    tl.sfin.contrib = sq.contrib;
                    tl.sfin.n0 = fc_shadow_counts(fcd);  // level 0's count: the first term
                    tl.sfin.fp = fp;
                    tl.sfin.tiles = sl->tiles.p;
                    tl.sfin.fo = fo;
                    tl.sfin.levels = tl.count_terms;
                    if (shadow_final_all)
                        for (int L = 1; L < tl.count_terms && L < kMaxLevels; ++L) tl.sfin.colors[L] = sl->n_color[L]->p;
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
        if (hx == kHostKernel) {  // this slot's final pixels -> the page-locked host framebuffer, now
            PGRT_REQUIRE(fs->out_mode == 0 && fs->out == fs->host_src, PGRT_ERR_INVALID_ARGUMENT,
                         "internal: host export of a frame that is not rendered into its staging framebuffer");
            launch_export_tiles(sl->tiles.p, nt, fs->host_src, fs->host_map, fs->ox, fs->oy, fs->pitch,
                                fs->frame_stride, s);
            debug_sync(s, "host export", 0, 0);
        }
        sl->host_fc.resize(batches);
        // the frame's counters to pinned host memory, zeroed on the device for the next frame
        launch_export_counters(sl->fc.p, sl->pinned_fc, batches, fs->deep_rec ? sl->tile_deep.p : nullptr,
                               sl->pinned_deep, nt, s);
        debug_sync(s, "export", 0, 0);
        PGRT_HIP(hipEventRecord(sl->ev_done, s));
    }
    if (fs->host_dst && hx == kHostOnce && K > 0) {  // one copy after every slot, on slot 0's stream
        FrameSlot* s0 = fs->slots[0].get();
        for (int j = 1; j < K; ++j) PGRT_HIP(hipStreamWaitEvent(s0->stream, fs->slots[j]->ev_done, 0));
        PGRT_HIP(hipMemcpyAsync(fs->host_dst, fs->host_src, fs->host_bytes, hipMemcpyDeviceToHost, s0->stream));
        PGRT_HIP(hipEventRecord(s0->ev_done, s0->stream));
    }
    if (hx == kHostSplit) {  // after every slot: a blit kernel's share on host_aux beside one DMA copy
#ifndef PGRT_HOST_SPLIT_PCT
#define PGRT_HOST_SPLIT_PCT 50
#endif
        FrameSlot* s0 = fs->slots[0].get();
        for (int j = 1; j < K; ++j) PGRT_HIP(hipStreamWaitEvent(s0->stream, fs->slots[j]->ev_done, 0));
        if (!fs->host_aux) {
            PGRT_HIP(hipStreamCreateWithFlags(&fs->host_aux, hipStreamNonBlocking));
            PGRT_HIP(hipEventCreateWithFlags(&fs->ev_host0, hipEventDisableTiming));
            PGRT_HIP(hipEventCreateWithFlags(&fs->ev_host1, hipEventDisableTiming));
        }
        const size_t kb = fs->host_bytes * PGRT_HOST_SPLIT_PCT / 100 / 256 * 256;  // 256-B aligned share
        PGRT_HIP(hipEventRecord(fs->ev_host0, s0->stream));
        PGRT_HIP(hipStreamWaitEvent(fs->host_aux, fs->ev_host0, 0));
        launch_blit_host(fs->host_src, fs->host_map, kb, fs->host_aux);
        PGRT_HIP(hipEventRecord(fs->ev_host1, fs->host_aux));
        if (kb < fs->host_bytes)
            PGRT_HIP(hipMemcpyAsync(reinterpret_cast<char*>(fs->host_dst) + kb,
                                    reinterpret_cast<const char*>(fs->host_src) + kb, fs->host_bytes - kb,
                                    hipMemcpyDeviceToHost, s0->stream));
        PGRT_HIP(hipStreamWaitEvent(s0->stream, fs->ev_host1, 0));
        PGRT_HIP(hipEventRecord(s0->ev_done, s0->stream));
    }
    PGRT_HIP(hipGetLastError());
    fs->stats.trace_launches = trace_launches;
    fs->stamp_used = slog.used;
    fs->stamp_overflow = slog.overflow;
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
        // the shadow queue's grid hint: the levels below the subtree launch only (the subtree
        // traces its own shadow rays; fc_shadow still counts them for the statistics)
        int shadow_need = 0;
        const int shadow_levels = sl->sub_first > 0 ? sl->sub_first : kMaxLevels;
        for (auto& h : sl->host_fc) {
            int sc = 0;
            for (int L = 0; L < shadow_levels; ++L) sc += fc_shadow(h, L);
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
    collect_timeline(ctx, fs);
}

// complete a pending frame: collect, gather (distributed), release the set's buffers
void finish_frame(pgrt_ctx* ctx, FrameSet* fs) {
    fs->pending = false;
    collect_frame(ctx, fs);  // a distributed frame's gather was queued at submission
    // a distributed frame's set is free once its own gather has read the tiles: gather_end recorded
    // ev_ready right behind it (also after a re-render's gather).  Recording it here again would put
    // the gathers of every frame submitted since in front of the set's next frame -- the frames in
    // flight would drain before each distributed call could start.
    if (!fs->distributed) PGRT_HIP(hipEventRecord(fs->ev_ready, ctx->stream));
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
                 int out_mode, int ox, int oy, int pitch, bool distributed, float* fb, int nframes,
                 long long frame_stride, TileDeal deal, bool defer_gather) {
    check_frame(ctx, p);
    if (distributed) check_comm(ctx);
    PGRT_REQUIRE(nframes >= 1 && nframes <= kMaxFramesPerCall, PGRT_ERR_INVALID_ARGUMENT,
                 "frames per call must be in [1, 64]");
    PGRT_REQUIRE(!fs->host_dst || (!distributed && out == fs->host_src && out_mode == 0), PGRT_ERR_INVALID_ARGUMENT,
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
    fs->poison = false;
    if (distributed) {
        // this rank's tiles of every frame, frame-major (the gather's layout, unpack_layout)
        fs->deal = deal;
        fs->gather_seq = ++ctx->gather_count;
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
                  int out_mode, int ox, int oy, int pitch, pgrt_stats* st, int nframes,
                  long long frame_stride, float* host_out, size_t host_bytes) {
    drain_frames(ctx);
    FrameSet* fs = frame_set(ctx, 0);
    // host_out: the framebuffer `out` (device) also lands in host memory of the same layout
    set_host_output(fs, host_out, out, host_bytes);
    PGRT_HIP(hipEventRecord(fs->ev_ready, ctx->stream));  // prior context-stream work first
    start_frame(ctx, fs, p, tiles, out, out_mode, ox, oy, pitch, false, nullptr, nframes, frame_stride);
    finish_frame(ctx, fs);
    if (st) *st = fs->stats;
}

// The host destination of fs's frames (NULL: none).  Page-locked memory (hipHostMalloc /
// hipHostRegister: it has a device-visible address) is written by the per-slot export kernels;
// pageable memory by one SDMA copy of `bytes` after the frame.
void set_host_output(FrameSet* fs, float* dst, float* src, size_t bytes) {
    fs->host_dst = dst;
    fs->host_src = dst ? src : nullptr;
    fs->host_bytes = dst ? bytes : 0;
    fs->host_map = nullptr;
    if (!dst) return;
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, dst, 0) == hipSuccess && dev)
        fs->host_map = static_cast<float*>(dev);
    else
        (void)hipGetLastError();  // not page-locked: the copy path
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

}  // namespace pgrt
