// context.cpp -- the C ABI core of libpgrt (include/pgrt.h): contexts, configuration, scene and
// camera, synchronous / asynchronous / batched renders, host-output frames, batch ray queries
// (rtcIntersect1 / rtcOccluded1 analogues) and the progressive frame sink.  The frame state and
// the other translation units are listed in context.hpp.
#include <thread>

#include "context.hpp"

using namespace pgrt;

// =========================================================================== C ABI

extern "C" {

const char* pgrt_version(void) { return "pgrt 0.3.0 (gfx950, abi 3)"; }

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
    ctx->cfg.size = sizeof(pgrt_config);
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
    if (!ctx->comm_aborted.empty() && ctx->stream) {
        // the communicator was aborted with a receive pending on this stream: the abort ends it,
        // but never wait for that without a bound -- if the stream has not drained after 10 s the
        // context's memory is left behind rather than the caller hung in the destructor
        const auto t0 = std::chrono::steady_clock::now();
        while (hipStreamQuery(ctx->stream) == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) return;
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    }
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    delete ctx;
}

const char* pgrt_last_error(const pgrt_ctx* ctx) { return ctx ? ctx->err.c_str() : "NULL context"; }

int pgrt_get_config(const pgrt_ctx* ctx, pgrt_config* cfg) {
    if (!ctx || !cfg) return PGRT_ERR_INVALID_ARGUMENT;
    *cfg = ctx->cfg;
    cfg->size = sizeof(pgrt_config);
    return PGRT_OK;
}

int pgrt_set_config(pgrt_ctx* ctx, const pgrt_config* cfg) {
    if (!ctx || !cfg) return PGRT_ERR_INVALID_ARGUMENT;
    return guarded(ctx, [&] {
        PGRT_REQUIRE(cfg->size == sizeof(pgrt_config), PGRT_ERR_INVALID_ARGUMENT,
                     "pgrt_config.size is " + std::to_string(cfg->size) + ", this library's pgrt_config has " +
                         std::to_string(sizeof(pgrt_config)) + " bytes (abi " + std::to_string(PGRT_ABI_VERSION) +
                         "): start from pgrt_get_config");
        PGRT_REQUIRE(cfg->host_export >= -1 && cfg->host_export <= 2, PGRT_ERR_INVALID_ARGUMENT,
                     "host_export must be 0, PGRT_HOST_EXPORT_KERNEL, PGRT_HOST_EXPORT_COPY or PGRT_HOST_EXPORT_SPLIT");
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
        PGRT_REQUIRE(cfg->peer_wait_ms >= 0, PGRT_ERR_INVALID_ARGUMENT, "peer_wait_ms must be >= 0 (0 = default)");
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
        const size_t bytes = (size_t)w * h * 4 * sizeof(float);
        if (ctx->group) {
            group_render(ctx, p, 1, ctx->out_tmp.p, st);
            PGRT_HIP(hipMemcpyAsync(rgba_host, ctx->out_tmp.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
        } else {
            // the frame's slots move their finished tiles to rgba_host themselves (set_host_output:
            // export kernels into page-locked memory, else one copy after the frame)
            render_tiles(ctx, p, rect_tiles(x, y, w, h), ctx->out_tmp.p, 0, x, y, w, st, 1, 0, rgba_host, bytes);
        }
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
        set_host_output(fs, nullptr, nullptr, 0);
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
            if (rgba_host) {
                fs->host_stage.alloc((size_t)nframes * w * h * 4);
                rgba_device = fs->host_stage.p;
                set_host_output(fs, rgba_host, fs->host_stage.p, (size_t)nframes * w * h * 4 * sizeof(float));
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
        if (!fs) check_comm(ctx);  // a distributed frame dropped when its communicator was aborted
        PGRT_REQUIRE(fs, PGRT_ERR_INVALID_ARGUMENT, "unknown ticket (or its frame set was reused)");
        finish_through(ctx, ticket);
        PGRT_HIP(hipEventSynchronize(fs->ev_ready));
        gather_times(fs, &fs->stats);
        if (st) *st = fs->stats;
    });
}

}  // extern "C"
