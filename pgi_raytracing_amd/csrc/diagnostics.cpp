// diagnostics.cpp -- the device-stamped launch timeline (pgrt_timeline_*: every frame kernel stamps
// its waves' start and end, stamps.hpp), the per-level frame diagnostics (pgrt_frame_diag) and the
// device math self-tests used by the parity tests.
#include "context.hpp"

using namespace pgrt;

namespace pgrt {
namespace {
thread_local StampLog* t_stamp_log = nullptr;
}
void set_stamp_log(StampLog* log) { t_stamp_log = log; }
StampLog* stamp_log() { return t_stamp_log; }

// the call's launch timeline: (first wave start, last wave end) and wave-duration percentiles per launch
void collect_timeline(pgrt_ctx* ctx, FrameSet* fs) {
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
    if (fs->stamp_overflow) {  // launches past the buffer were not stamped: say so in the records
        pgrt_timeline_rec r{fs->ticket, 0, PGRT_TL_DROPPED, -1, 0, 0, 0, 0, 0, 0, 0};
        ctx->timeline.push_back(r);
        fs->stamp_overflow = false;
    }
}

}  // namespace pgrt

extern "C" {

int pgrt_timeline_enable(pgrt_ctx* ctx, int on) {
    if (!ctx) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        drain_frames(ctx);  // pending frames were enqueued with the old choice
        ctx->timeline_on = on != 0;
        if (!ctx->timeline_on)  // the stamp buffers (64 MB per frame set) go with the timeline
            for (auto& fs : ctx->sets) fs->stamps.release();
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
