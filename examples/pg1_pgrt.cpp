// pg1_pgrt.cpp -- the reference's entry point (APP/pg1_embree.cpp:4-22) on libpgrt.
//
//   pg1_pgrt tutorial_1                 tutorials.cpp:142-167 (single-triangle closest hit)
//   pg1_pgrt render <obj> <env> <out.raw> [W H S d dof]
//                                        raytrace_loop (tutorials.cpp:181-200): the default pose,
//                                        one GPU frame, RGBA float32 written raw (+ .pfm)
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

int main(int argc, char** argv) {
    std::printf("PG1 on MI355X (libpgrt %s)\n\n", pgrt_version());
    try {
        if (argc >= 2 && std::string(argv[1]) == "tutorial_1") return tutorial_1();
        if (argc >= 2 && std::string(argv[1]) == "render") return render(argc, argv);
    } catch (const pgrt::Exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
    std::fprintf(stderr, "usage: %s tutorial_1 | render <obj> <env> <out.raw> [W H S d dof]\n", argv[0]);
    return 2;
}
