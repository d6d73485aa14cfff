// tail.hip -- the deep levels of the Whitted recursion (raytracer.cpp:237-394, trace() called
// for the children of dielectric hits, :306-316) as ONE persistent launch with device-side level
// iteration.
//
// Per level, the wavefront pipeline (render.hip) waits for the slowest ray of a level before the
// next level starts: the deep levels of C2 hold a few ten thousand rays each, and every launch
// lasts as long as its slowest ray's dependent chain of BVH fetches, so the last frames of a
// burst pay the sum of those floors.  Here the levels overlap: a block claims up to 256 rays of
// the shallowest level with unclaimed rays, traces them (one lane per ray, stack in LDS), shades
// them with the same phases as k_shade (shade_ray.hpp) and hands each child to the next level
// the moment it is written.  A ray's time on the chain is then its own ancestors' chain, not the
// sum of every level's slowest ray.
//
// Hand-off (gfx950: 8 XCDs with private L2s, MI355X_MICROARCH.md / cdna_hip_programming.md
// Guideline 16): a child is 5 words of 8 bytes -- (org.xy) (org.z, tnear) (dir.xy) (dir.z, tfar)
// (medium bits, epoch) -- written by relaxed agent-scope atomic stores (write-through `sc1`),
// the payload words drained (`s_waitcnt vmcnt(0)`) before the last word, whose high half is the
// batch's epoch: the slot's ready flag.  The consumer polls that word relaxed and reads the
// payload with relaxed agent-scope loads (`sc1`, never through a stale L1).  Epochs count up per
// batch and slot (never 0), so no flag needs clearing.  Every wait is bounded: a wait that runs
// out sets FrameCounters::tail_err and the frame fails loudly instead of hanging the GPU.
//
// Termination: rays are claimed only below a level's current count (slots already allocated by a
// running producer, which writes them without waiting on anything), and a block leaves when the
// rays shaded so far (tail_done, counted after their children were allocated) equal the rays
// allocated on every tail level -- then no ray is in flight and none can appear.
#include "shade_ray.hpp"
#include "traverse.hpp"

namespace pgrt {

constexpr int kTailBlock = 256;
// bounded waits, in wall-clock ticks (wall_clock64: 100 MHz): far beyond any real hand-off
constexpr long long kTailWaitTicks = 20000000;  // 0.2 s
// idle blocks (no unclaimed ray right now) leave once the others can take every ray that may yet
// appear, but at least this many stay: every idle poller loads the counters the producers update
constexpr int kTailKeep = 32;

namespace {

typedef unsigned long long u64;
constexpr int kRlx = __ATOMIC_RELAXED;

__device__ __forceinline__ u64 gload(const u64* p) {
    return __hip_atomic_load(const_cast<u64*>(p), kRlx, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(u64* p, u64 v) { __hip_atomic_store(p, v, kRlx, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int iload(const int* p) {
    return __hip_atomic_load(const_cast<int*>(p), kRlx, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 pack2(float a, float b) {
    return (u64)__float_as_uint(a) | ((u64)__float_as_uint(b) << 32);
}
__device__ __forceinline__ float lo_f(u64 v) { return __uint_as_float((unsigned)(v & 0xffffffffull)); }
__device__ __forceinline__ float hi_f(u64 v) { return __uint_as_float((unsigned)(v >> 32)); }

// payload of one child (4 words), then -- after the caller drained the stores -- its flag word
__device__ __forceinline__ void put_payload(u64* g, float4 o, float4 d) {
    gstore(g, pack2(o.x, o.y));
    gstore(g + 1, pack2(o.z, o.w));
    gstore(g + 2, pack2(d.x, d.y));
    gstore(g + 3, pack2(d.z, d.w));
}
__device__ __forceinline__ void put_flag(u64* g, float medium, unsigned epoch) {
    gstore(g + 4, (u64)__float_as_uint(medium) | ((u64)epoch << 32));
}

// rays of tail level l that exist (allocated and inside its queue)
__device__ __forceinline__ int level_avail(const TailLaunch& t, int l) {
    const int c = l == t.first ? fc_count(*t.fc, l)
                               : (int)(unsigned)(__hip_atomic_load(&t.fc->alloc[l - 1], kRlx, __HIP_MEMORY_SCOPE_AGENT) &
                                                 0xffffffffull);
    return min(c, t.cap[l]);
}

}  // namespace

template <bool LDS_TABLES>
__global__ __launch_bounds__(kTailBlock) void k_tail(SceneView s, FrameParams fp, TailLaunch t) {
    extern __shared__ int lstack[];  // traversal stacks: [depth + 2][kTailBlock]
    __shared__ float lut255[256];
    __shared__ DevMaterial smat[LDS_TABLES ? kLdsMats : 1];
    __shared__ DevTexture stex[LDS_TABLES ? kLdsTex : 1];
    __shared__ ShadeAllocLds<kTailBlock> alds;
    __shared__ int pick[4];  // level, first slot, end slot, status (0 work, 1 idle, 2 done, 3 error, 4 leave,
                         // 5 empty ticket)
    if constexpr (LDS_TABLES) {
        for (int k = threadIdx.x; k < s.nmat; k += kTailBlock) smat[k] = s.mats[k];
        for (int k = threadIdx.x; k < s.ntex; k += kTailBlock) stex[k] = s.tex[k];
        s.tex = stex;
    }
    const DevMaterial* mats = LDS_TABLES ? smat : s.mats;
    fill_byte_lut(lut255);
    FrameCounters* fc = t.fc;
    const int tid = threadIdx.x;
    const int sbits = s.nlight > 0 ? 32 - __clz(s.nlight) : 0;
    // every tail level's shadow rays follow those of the levels before the tail (final by now)
    int sq_base = 0;
    for (int l = 0; l < t.first; ++l) sq_base += fc_shadow(*fc, l);
    unsigned long long* const shadow_ctr = &fc->alloc[t.first];
    int it_par = 0, idle = 0;
    long long idle_since = 0;
    if (tid == 0) atomicAdd(&fc->tail_alive, 1);
    // profile == 2: where the launch's time goes (FrameCounters::trav[first][8..13], diag only):
    // block iterations, idle polls, flag polls of waiting lanes, and thread 0's cycles / 1024 in
    // the claim, in loading + tracing, in shading + hand-off
    unsigned long long st_iter = 0, st_idle = 0, st_pick = 0, st_trace = 0, st_shade = 0;
    long long c0 = 0;
    for (;;) {
        if (fp.count && tid == 0) c0 = clock64();
        if (tid == 0) {
            int L = -1, lo = 0, hi = 0, status = 1;
            // tail_done first, then the counts: done == allocated means nothing is in flight
            const int done = iload(&fc->tail_done);
            long long total = 0;
            for (int l = t.first; l < t.levels; ++l) {
                const int c = level_avail(t, l);
                total += c;
                // claim 256 slots of the shallowest level with unclaimed rays: a fetch-add ticket
                // (a CAS loop over 1024 contending blocks costs O(blocks^2) atomics)
                if (L < 0 && iload(&fc->tail_head[l]) < c) {
                    L = l;
                    lo = atomicAdd(&fc->tail_head[l], kTailBlock);
                    hi = lo + kTailBlock;
                    status = 0;
                }
            }
            if (L < 0 && done >= total) status = 2;
            if (L < 0 && status == 1) {
                // idle: leave when the blocks still running can take every ray that may yet appear
                // (each ray in flight has at most 2 children; their children come later still)
                const long long inflight = total - done;
                if ((long long)(iload(&fc->tail_alive) - kTailKeep) * kTailBlock > 4 * inflight) {
                    if (atomicAdd(&fc->tail_alive, -1) > kTailKeep) status = 4;
                    else atomicAdd(&fc->tail_alive, 1);
                }
            }
            if (status == 0) {
                // a ticket can run ahead of the level's rays (another block took the last ones
                // first): wait until they exist, or until the level is closed -- every ray of the
                // levels before it shaded, so its count is final -- and keep the slots below it
                const long long w0 = wall_clock64();
                int back = 0;
                for (;;) {
                    const int c = level_avail(t, L);
                    if (c >= hi) break;
                    bool closed = true;
                    for (int l = t.first; l < L && closed; ++l) {
                        const int dl = iload(&fc->tail_done_level[l]);  // done before count: see tail_done
                        closed = dl >= level_avail(t, l);
                    }
                    if (closed && level_avail(t, L) < hi) {
                        hi = max(lo, level_avail(t, L));
                        break;
                    }
                    if (wall_clock64() - w0 > kTailWaitTicks) {
                        atomicOr(&fc->tail_err, 4);
                        hi = lo;
                        break;
                    }
                    for (int k = 0, n = min(++back, 8); k < n; ++k) __builtin_amdgcn_s_sleep(16);
                }
                if (hi <= lo) status = 5;  // nothing left under the ticket: claim again
            }
            if (iload(&fc->tail_err)) status = 3;
            pick[0] = L;
            pick[1] = lo;
            pick[2] = hi;
            pick[3] = status;
        }
        __syncthreads();
        const int L = pick[0], lo = pick[1], hi = pick[2], status = pick[3];
        __syncthreads();
        if (fp.count && tid == 0) {
            const long long c1 = clock64();
            st_pick += (unsigned long long)(c1 - c0);
            c0 = c1;
            if (status == 1) ++st_idle;
            if (status == 0) ++st_iter;
        }
        if (status == 5) continue;
        if (status >= 2) break;
        if (status == 1) {  // back off: each poll loads the counters the producing blocks update
            if (idle == 0) idle_since = wall_clock64();
            else if (wall_clock64() - idle_since > kTailWaitTicks) {
                if (tid == 0) atomicOr(&fc->tail_err, 1);
                break;
            }
            for (int k = 0, n = min(++idle, 8); k < n; ++k) __builtin_amdgcn_s_sleep(32);
            continue;
        }
        idle = 0;
        const int i = lo + tid;
        const bool active = i < hi;
        float4 o4 = make_float4(0, 0, 0, 0), d4 = make_float4(0, 0, 1, -1.0f);
        float rtime = 0.0f;
        if (active) {
            if (L == t.first) {  // written by the previous launch (the shade of level first - 1)
                o4 = t.q_first.ro[i];
                d4 = t.q_first.rd[i];
                rtime = t.q_first.time[i];
            } else {  // handed over inside this launch: poll the flag word, then read the payload
                const u64* g = t.gran[L] + 5 * (size_t)i;
                u64 f = gload(g + 4);
                if ((unsigned)(f >> 32) != t.epoch) {
                    const long long w0 = wall_clock64();
                    unsigned polls = 0;
                    while ((unsigned)(f >> 32) != t.epoch && wall_clock64() - w0 < kTailWaitTicks) {
                        __builtin_amdgcn_s_sleep(2);
                        f = gload(g + 4);
                        ++polls;
                    }
                    if (fp.count) atomicAdd(&fc->trav[t.first][10], (unsigned long long)(polls + 15) / 16);  // x16
                }
                if ((unsigned)(f >> 32) == t.epoch) {
                    const u64 w0 = gload(g), w1 = gload(g + 1), w2 = gload(g + 2), w3 = gload(g + 3);
                    o4 = make_float4(lo_f(w0), hi_f(w0), lo_f(w1), hi_f(w1));
                    d4 = make_float4(lo_f(w2), hi_f(w2), lo_f(w3), hi_f(w3));
                    rtime = lo_f(f);
                } else {
                    atomicOr(&fc->tail_err, 2);  // never handed over: the frame fails loudly
                }
            }
        }
        const float4 h = trace_closest_lds(s, o4, d4, lstack, kTailBlock, tid);
        if (fp.count) {
            __syncthreads();  // (profile only) thread 0 times the block's slowest trace
            if (tid == 0) {
                const long long c1 = clock64();
                st_trace += (unsigned long long)(c1 - c0);
                c0 = c1;
            }
        }
        ShadeOut r;
        shade_eval(s, mats, lut255, L, fp.max_level, active, o4, d4, rtime, h, r);
        // children counted on fc->alloc[L] (the next level's count), shadow rays on alloc[first]
        const ShadeSlots sl = shade_alloc_end<kTailBlock>(
            alds, it_par, sq_base,
            shade_alloc_begin<kTailBlock>(alds, it_par, fc, L, sbits, r, &fc->alloc[L], shadow_ctr));
        if (active) {
            int4 link = make_int4(-1, -1, -1, 0);
            if (r.kind == 1) {
                const int nl = L + 1;
                if (nl >= t.levels || (r.nchild == 2 ? max(sl.refl, sl.refr) : sl.refl) >= t.cap[nl]) {
                    atomicOr(&fc->overflow, 1);  // re-rendered with larger queues
                } else {
                    u64* g0 = t.gran[nl] + 5 * (size_t)sl.refl;
                    put_payload(g0, child_org(r), child_dir(r.refl_dir));
                    u64* g1 = r.nchild == 2 ? t.gran[nl] + 5 * (size_t)sl.refr : nullptr;
                    if (g1) put_payload(g1, child_org(r), child_dir(r.refr_dir));
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // payload visible before its flag
                    put_flag(g0, r.n1, t.epoch);
                    if (g1) put_flag(g1, r.n2, t.epoch);
                    link.x = sl.refl;
                    link.y = g1 ? sl.refr : -1;
                }
            }
            emit_node(s, mats, i, r, sl, link, t.nodes[L], t.sq, fc);
        }
        __syncthreads();  // every ray of the batch shaded and its children allocated
        if (tid == 0) {
            atomicAdd(&fc->tail_done_level[L], hi - lo);
            atomicAdd(&fc->tail_done, hi - lo);
        }
        if (fp.count && tid == 0) st_shade += (unsigned long long)(clock64() - c0);
    }
    if (fp.count && tid == 0) {
        unsigned long long* d = fc->trav[t.first];
        atomicAdd(&d[8], st_iter);
        atomicAdd(&d[9], st_idle);
        atomicAdd(&d[11], st_pick >> 10);
        atomicAdd(&d[12], st_trace >> 10);
        atomicAdd(&d[13], st_shade >> 10);
    }
    // (a block leaving at termination or on an error keeps its place in tail_alive: idle blocks
    // only ever compare it with kTailKeep)
}

bool tail_available(const SceneView& s) {
    return !s.wide && s.root >= 0 && (size_t)(s.depth + 2) * kTailBlock * sizeof(int) <= 65536;
}

void launch_tail(const SceneView& s, const FrameParams& fp, const TailLaunch& t, hipStream_t stream) {
    const size_t lds = (size_t)(s.depth + 2) * kTailBlock * sizeof(int);
    const bool tables = s.nmat <= kLdsMats && s.ntex <= kLdsTex;
    if (tables)
        hipLaunchKernelGGL(k_tail<true>, dim3(t.grid), dim3(kTailBlock), lds, stream, s, fp, t);
    else
        hipLaunchKernelGGL(k_tail<false>, dim3(t.grid), dim3(kTailBlock), lds, stream, s, fp, t);
}

}  // namespace pgrt
