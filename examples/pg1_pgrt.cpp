// pg1_pgrt.cpp -- the reference's entry point (APP/pg1_embree.cpp:4-22) on libpgrt.
//
//   pg1_pgrt tutorial_1                 tutorials.cpp:142-167 (single-triangle closest hit)
//   pg1_pgrt render <obj> <env> <out.raw> [W H S d dof]
//                                        raytrace_loop (tutorials.cpp:181-200): the default pose,
//                                        one GPU frame, RGBA float32 written raw (+ .pfm)
//   pg1_pgrt bench <obj> <env> [steps warmup frames_per_call in_flight]
//                                        bench.py's C2 line through this C++ drop-in (one JSON line)
#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <memory>
#include <vector>

#include "pgrt_raytracer.hpp"

static int tutorial_1() {
    // add_triangle (tutorials.cpp:29-80) through the scene ABI
    const float pos[9] = {0, 0, 0, 2, 0, 0, 0, 3, 0};
    const float nrm[9] = {0, 0, 1, 0, 0, 1, 0, 0, 1};
    const float uv[6] = {0, 1, 1, 1, 0, 0};
    const int mat_id[1] = {0};
    pgrt_material m{{0.4f, 0.4f, 0.4f}, {0.8f, 0.8f, 0.8f}, 1.0f, 1.5f, 0, -1};
    pgrt_scene_desc d{};
    d.num_triangles = 1;
    d.positions = pos;
    d.normals = nrm;
    d.uvs = uv;
    d.material_ids = mat_id;
    d.num_materials = 1;
    d.materials = &m;
    d.env_texture = -1;
    pgrt_ctx* ctx = nullptr;
    pgrt::check(nullptr, pgrt_create(0, &ctx), "pgrt_create");
    pgrt::check(ctx, pgrt_set_scene(ctx, &d), "pgrt_set_scene");
    // generate_and_trace_ray (tutorials.cpp:83-139)
    const float ray[8] = {0.1f, 0.2f, 2.0f, FLT_MIN, 0.0f, 0.0f, -1.0f, FLT_MAX};
    float hit[4];
    pgrt::check(ctx, pgrt_intersect_closest(ctx, ray, 1, hit), "pgrt_intersect_closest");
    int prim;
    std::memcpy(&prim, &hit[3], 4);
    if (prim >= 0) {
        const float u = hit[1], v = hit[2], w = 1.0f - u - v;
        float n[3], tc[2];
        for (int k = 0; k < 3; ++k) n[k] = std::fma(w, nrm[k], std::fma(u, nrm[3 + k], v * nrm[6 + k]));
        for (int k = 0; k < 2; ++k) tc[k] = std::fma(w, uv[k], std::fma(u, uv[2 + k], v * uv[4 + k]));
        std::printf("normal = (%0.3f, %0.3f, %0.3f)\n", n[0], n[1], n[2]);
        std::printf("tex_coord = (%0.3f, %0.3f)\n", tc[0], tc[1]);
    }
    pgrt_destroy(ctx);
    return EXIT_SUCCESS;
}

static int render(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s render <obj> <env> <out.raw> [W H S d dof [devices]]\n", argv[0]);
        return 2;
    }
    const int W = argc > 5 ? std::atoi(argv[5]) : 640, H = argc > 6 ? std::atoi(argv[6]) : 480;
    // optional 11th argument: HIP devices "0,1,..." -> one process renders on all of them
    std::vector<int> devices;
    if (argc > 10)
        for (const char* q = argv[10]; *q;) {
            devices.push_back(std::atoi(q));
            while (*q && *q != ',') ++q;
            if (*q == ',') ++q;
        }
    const pgrt::Vector3 from(-140.0f, -175.0f, 80.0f), at(0.0f, 0.0f, 40.0f);
    std::unique_ptr<pgrt::Raytracer> rt =
        devices.empty() ? std::make_unique<pgrt::Raytracer>(W, H, pgrt::deg2rad(42.185f), from, at)
                        : std::make_unique<pgrt::Raytracer>(W, H, pgrt::deg2rad(42.185f), from, at, devices);
    pgrt::Raytracer& raytracer = *rt;
    raytracer.LoadScene(argv[2], argv[3]);
    auto& p = raytracer.params();
    p.spp_side = argc > 7 ? std::atoi(argv[7]) : 3;
    p.max_level = argc > 8 ? std::atoi(argv[8]) : 7;
    p.dof = argc > 9 ? std::atoi(argv[9]) : 1;
    p.jitter = (p.spp_side > 1 || p.dof) ? PGRT_JITTER_HASH : PGRT_JITTER_NONE;
    auto t0 = std::chrono::steady_clock::now();
    pgrt_stats st = raytracer.Render();
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const unsigned long long rays = st.rays_primary + st.rays_shadow + st.rays_reflect + st.rays_refract;
    std::printf("Surfaces = %d\nMaterials = %d\n", raytracer.surfaces(), raytracer.materials());
    std::printf("%dx%d S=%d d=%d dof=%d: %.3f ms, %llu rays (%.1f Mrays/s)\n", W, H, p.spp_side, p.max_level,
                p.dof, ms, rays, rays / ms * 1e-3);
    FILE* f = std::fopen(argv[4], "wb");
    if (!f) return 1;
    std::fwrite(raytracer.frame().data(), sizeof(float), raytracer.frame().size(), f);
    std::fclose(f);
    pgrt::write_pfm((std::string(argv[4]) + ".pfm").c_str(), raytracer.frame().data(), W, H);
    return EXIT_SUCCESS;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static unsigned long long rays_of(const pgrt_stats& st) {
    return st.rays_primary + st.rays_shadow + st.rays_reflect + st.rays_refract;
}

// bench.py's C2 line (1920x1080, S = 1, d = 5, pinhole, distinct frames: hash jitter keyed by the
// frame index; calls of F frames, `in_flight` calls in flight, device framebuffers, untimed set-up
// of one call per slot, then `warmup` untimed and `steps` timed frames), the synchronous frame
// latency (one frame in flight, pgrt_render_device), and the reference's own default frame
// (raytracer.cpp:398-400, tutorials.cpp:186-191: 640x480, S = 3 thin lens, d = 7) to host memory
// as Raytracer::Render does it (median of 10 after 2).  Everything goes through the facade the
// drop-in uses (including its GPU_MAX_HW_QUEUES preference).
static int bench(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s bench <obj> <env> [steps warmup frames_per_call in_flight]\n", argv[0]);
        return 2;
    }
    const int steps = argc > 4 ? std::atoi(argv[4]) : 20, warmup = argc > 5 ? std::atoi(argv[5]) : 5;
    const int F = argc > 6 ? std::atoi(argv[6]) : 8, in_flight = argc > 7 ? std::atoi(argv[7]) : 8;
    const pgrt::Vector3 from(-140.0f, -175.0f, 80.0f), at(0.0f, 0.0f, 40.0f);
    const int W = 1920, H = 1080;
    double ms_per_frame = 0, latency_ms = 0, mrays = 0;
    unsigned long long rays_total = 0;
    {
        pgrt::Raytracer rt(W, H, pgrt::deg2rad(42.185f), from, at);
        rt.LoadScene(argv[2], argv[3]);
        pgrt_render_params& p = rt.params();
        p.spp_side = 1;
        p.max_level = 5;
        p.dof = 0;
        p.jitter = PGRT_JITTER_HASH;
        p.frame = 0;
        const size_t call_bytes = (size_t)F * W * H * 16;
        void* fb = nullptr;
        pgrt::check(rt.context(), pgrt_device_alloc(rt.context(), call_bytes * in_flight, &fb), "pgrt_device_alloc");
        rt.SetFramesInFlight(in_flight);
        int call = 0;
        auto run = [&](int n) {
            std::vector<unsigned long long> pending;
            unsigned long long rays = 0;
            for (int done = 0; done < n;) {
                const int nf = std::min(F, n - done);
                pending.push_back(rt.SubmitFrames(nf, static_cast<char*>(fb) + (size_t)(call++ % in_flight) * call_bytes));
                done += nf;
                if ((int)pending.size() >= in_flight) {
                    rays += rays_of(rt.Wait(pending.front()));
                    pending.erase(pending.begin());
                }
            }
            for (unsigned long long t : pending) rays += rays_of(rt.Wait(t));
            return rays;
        };
        run(in_flight * F);
        run(warmup);
        pgrt::check(rt.context(), pgrt_synchronize(rt.context()), "pgrt_synchronize");
        const double t0 = now_ms();
        rays_total = run(steps);
        pgrt::check(rt.context(), pgrt_synchronize(rt.context()), "pgrt_synchronize");
        const double el = now_ms() - t0;
        ms_per_frame = el / std::max(1, steps);
        mrays = rays_total / el * 1e-3;
        rt.SetFramesInFlight(1);
        std::vector<double> lat;
        for (int k = 0; k < std::min(steps, 30) + 2; ++k) {
            const double t1 = now_ms();
            pgrt_stats st{};
            pgrt::check(rt.context(), pgrt_render_device(rt.context(), &p, fb, &st), "pgrt_render_device");
            if (k >= 2) lat.push_back(now_ms() - t1);
        }
        std::sort(lat.begin(), lat.end());
        latency_ms = lat.empty() ? 0 : lat[lat.size() / 2];
        pgrt_device_free(rt.context(), fb);
    }
    // the reference's default frame, to host memory (Raytracer::Render = pgrt_render)
    pgrt::Raytracer ref(640, 480, pgrt::deg2rad(42.185f), from, at);
    ref.LoadScene(argv[2], argv[3]);
    std::vector<double> t_ref;
    unsigned long long ref_rays = 0;
    for (int k = 0; k < 12; ++k) {
        const double t1 = now_ms();
        const pgrt_stats st = ref.Render();
        if (k >= 2) t_ref.push_back(now_ms() - t1);
        ref_rays = rays_of(st);
    }
    std::sort(t_ref.begin(), t_ref.end());
    const double ref_ms = t_ref[t_ref.size() / 2];
    const char* hwq = std::getenv("GPU_MAX_HW_QUEUES");
    std::printf("{\"workload\": \"C2 1920x1080 d=5 1 spp, distinct frames, through pgrt_raytracer.hpp\", "
                "\"ms_per_frame\": %.5f, \"mrays_per_s\": %.1f, \"rays\": %llu, \"steps\": %d, \"warmup\": %d, "
                "\"frames_per_call\": %d, \"in_flight\": %d, \"frame_latency_ms\": %.4f, "
                "\"reference_default_frame\": {\"width\": 640, \"height\": 480, \"spp_side\": 3, \"dof\": 1, "
                "\"max_level\": 7, \"ms_per_frame_host\": %.4f, \"rays_per_frame\": %llu, \"mrays_per_s\": %.1f}, "
                "\"GPU_MAX_HW_QUEUES\": \"%s\"}\n",
                ms_per_frame, mrays, rays_total, steps, warmup, F, in_flight, latency_ms, ref_ms, ref_rays,
                ref_rays / ref_ms * 1e-3, hwq ? hwq : "");
    return EXIT_SUCCESS;
}

int main(int argc, char** argv) {
    std::printf("PG1 on MI355X (libpgrt %s)\n\n", pgrt_version());
    try {
        if (argc >= 2 && std::string(argv[1]) == "tutorial_1") return tutorial_1();
        if (argc >= 2 && std::string(argv[1]) == "render") return render(argc, argv);
        if (argc >= 2 && std::string(argv[1]) == "bench") return bench(argc, argv);
    } catch (const pgrt::Exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
    std::fprintf(stderr, "usage: %s tutorial_1 | render <obj> <env> <out.raw> [W H S d dof] | bench <obj> <env>\n", argv[0]);
    return 2;
}
