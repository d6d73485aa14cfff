// distributed.cpp -- multi-GPU frames: image tiles dealt to ranks (tiles.hpp),
// every rank's tile-compact buffer gathered to rank 0 over RCCL (grouped ncclSend / ncclRecv on the
// context stream, queued behind the frame on the device) and unpacked there; the queue-overflow
// agreement (a flag at the tail of every rank's send); the single-process multi-device context
// (pgrt_create_devices); and the distributed C ABI.
#include <thread>

#include "context.hpp"

using namespace pgrt;

namespace pgrt {

void regather_rank0(pgrt_ctx* ctx, FrameSet* fs, bool own, const std::vector<int>& peers);

// a multi-process distributed frame whose gather goes over RCCL (the overflow flags ride along)
bool rccl_gather(const pgrt_ctx* ctx, const FrameSet* fs) {
    return fs->distributed && !ctx->emulated && fs->deal.world > 1 && ctx->comm != nullptr;
}

// Wait for fs's frame, re-render it after a queue overflow (larger queues), fill fs->stats.  A
// distributed frame's gather was queued with the frame (device-ordered, start_frame).  There is no
// control collective: the tail of every rank's send carries its overflow flag and the frame's
// sequence number (gather_begin).  A rank whose queues overflowed re-renders its tiles and sends
// them again; rank 0 reads the peers' tails (gather_end copies them to host memory behind the
// unpack), receives the flagged ranks' tiles again and unpacks them (and its own, when it
// overflowed).  The re-send / re-receive of a frame is posted when that frame is COLLECTED, so
// every rank must submit and wait for its distributed frames in the same order (the same calls of
// the same program, as bench.py's ranks do) -- point-to-point operations match in posting order.
// Rank 0 checks the sequence number of every tail it receives and fails loudly on a mismatch
// instead of unpacking another frame's tiles.  A rank that gives up after kMaxRetries re-renders
// still sends (flag 2, "poison"), so rank 0's receive completes and rank 0 fails too instead of
// waiting forever.  Non-zero ranks never wait for another rank; rank 0 waits for the frame's own
// gather only, and at most kPeerWaitSeconds (a rank that died without sending).
constexpr int kMaxRetries = 8;
// Rank 0's wait for the peers' tiles of one gather is bounded (pgrt_config.peer_wait_ms, default
// 120 s): a peer that died or never submitted the frame would leave rank 0's ncclRecv pending
// forever.  On timeout the communicator is aborted (abort_comm) and the caller gets PGRT_ERR_RCCL
// -- from this call, from every later distributed call, and pgrt_destroy still returns.
constexpr double kPeerWaitSeconds = 120.0;
double peer_wait_seconds(const pgrt_ctx* ctx) {
    return ctx->cfg.peer_wait_ms > 0 ? ctx->cfg.peer_wait_ms * 1e-3 : kPeerWaitSeconds;
}

// The peers' tiles did not arrive in time: ncclCommAbort (RCCL's kernels poll the communicator's
// abort flag, so the pending ncclRecv on the context stream ends and that stream drains), drop
// every frame still in flight (their gathers used the same communicator) and fail.  Later
// distributed calls fail at once (check_comm); pgrt_destroy does not wait on a stream that never
// drains (context.cpp).
[[noreturn]] void abort_comm(pgrt_ctx* ctx, const std::string& why) {
    if (ctx->comm) {
        (void)ncclCommAbort(ctx->comm);
        ctx->comm = nullptr;
    }
    ctx->comm_aborted = why;
    for (auto& s : ctx->sets)
        if (s->distributed) s->pending = false;
    throw Error(PGRT_ERR_RCCL, why);
}

void check_comm(const pgrt_ctx* ctx) {
    PGRT_REQUIRE(ctx->comm_aborted.empty(), PGRT_ERR_RCCL,
                 "the communicator was aborted (" + ctx->comm_aborted +
                     "); distributed frames need a new context or pgrt_comm_init");
}

// diagnostics only (tests/test_gpu_parity.py): PGRT_DEBUG_PEER_STALL=1 makes rank 0 of an
// emulated world (PGRT_EMULATE_RANK=0/N) behave as if its peers never sent: the bounded wait runs
// out and the abort path above is taken (one GPU cannot host a world-2 RCCL communicator)
bool debug_peer_stall() {
    static const bool on = [] {
        const char* e = getenv("PGRT_DEBUG_PEER_STALL");
        return e && e[0] == '1';
    }();
    return on;
}

// hipEventSynchronize with a time limit: spin on hipEventQuery for the first 2 ms (a frame's gather
// usually lands within it), then poll every 50 us; false on timeout
bool wait_event_bounded(hipEvent_t e, double seconds) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return true;
        if (q != hipErrorNotReady) PGRT_HIP(q);
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > seconds) return false;
        if (el > 2e-3) std::this_thread::sleep_for(std::chrono::microseconds(50));
        else std::this_thread::yield();
    }
}

// rank 0: the peers' tails of fs's gather have landed, or the communicator is aborted
void rank0_await_peers(pgrt_ctx* ctx, FrameSet* fs) {
    const double limit = peer_wait_seconds(ctx);
    bool ok;
    if (ctx->emulated) {  // the diagnostics stall: nothing was sent, wait out the limit
        std::this_thread::sleep_for(std::chrono::duration<double>(limit));
        ok = false;
    } else {
        ok = wait_event_bounded(fs->ev_flags, limit);
    }
    if (!ok)
        abort_comm(ctx, "rank 0 received no tiles of distributed frame " + std::to_string(fs->gather_seq) +
                            " within " + std::to_string(limit) +
                            " s: a rank failed or did not submit the frame (communicator aborted)");
}

void collect_frame(pgrt_ctx* ctx, FrameSet* fs) {
    int retries = 0;
    const bool rccl = rccl_gather(ctx, fs);
    if (fs->distributed && ctx->rank == 0 && ctx->emulated && fs->deal.world > 1 && debug_peer_stall())
        rank0_await_peers(ctx, fs);  // diagnostics: always times out
    for (;;) {
        const bool mine = read_frame_counters(ctx, fs);
        if (!rccl || ctx->rank != 0) {
            if (!mine) break;
            if (rccl && retries + 1 >= kMaxRetries) {  // give up, but keep rank 0's receive matched
                fs->poison = true;
                gather_frame(ctx, fs);
                throw Error(PGRT_ERR_OUT_OF_MEMORY, "ray queues kept overflowing (rank " + std::to_string(ctx->rank) +
                                                        " gave up; rank 0 is told by the poison flag of its send)");
            }
            rerender_frame(ctx, fs, true, retries);
            if (fs->distributed) gather_frame(ctx, fs);  // rank != 0: the tiles again, to rank 0
            continue;
        }
        rank0_await_peers(ctx, fs);
        std::vector<int> peers;
        {
            const int world = fs->deal.world;
            unsigned seqs[kMaxRanks];
            int regather[kMaxRanks], bad = -1;
            for (int r = 0; r < world; ++r) seqs[r] = (unsigned)fs->peer_flags[kMaxRanks + r];
            const int v = gather_tail_verdict(fs->peer_flags, seqs, world, fs->gather_seq, regather, &bad);
            PGRT_REQUIRE(v != -1, PGRT_ERR_RCCL,
                         "rank " + std::to_string(bad) + " sent the tiles of its distributed frame " +
                             std::to_string(bad >= 0 ? seqs[bad] : 0u) + " where rank 0 expected frame " +
                             std::to_string(fs->gather_seq) +
                             ": every rank must submit and wait for distributed frames in the same order");
            PGRT_REQUIRE(v != -2, PGRT_ERR_OUT_OF_MEMORY,
                         "rank " + std::to_string(bad) + " gave up on the frame: its ray queues kept overflowing");
            for (int r = 1; r < world; ++r)
                if (regather[r]) peers.push_back(r);
        }
        if (!mine && peers.empty()) break;
        if (mine) {
            rerender_frame(ctx, fs, true, retries);
        } else {
            PGRT_REQUIRE(++retries < kMaxRetries, PGRT_ERR_OUT_OF_MEMORY, "ray queues kept overflowing");
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
        f.poison = fs->poison ? 1 : 0;
        f.seq = fs->gather_seq;
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
    std::fill(fs->peer_flags, fs->peer_flags + 2 * kMaxRanks, 0);
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
        // (the set's ready event stays behind its own gather, gather_end: see finish_frame)
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
        set_host_output(fs, nullptr, nullptr, 0);
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

}  // namespace pgrt

extern "C" {

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
        ctx->comm_aborted.clear();
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
        set_host_output(fs, nullptr, nullptr, 0);
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

}  // extern "C"
