// scene.cpp -- pgrt_set_scene's work: host packing of the scene arrays and the on-device BVH
// build (replaces Raytracer::LoadScene's Embree upload, APP/raytracer.cpp:48-128), and the
// PinHoleCamera constructor (APP/PinHoleCamera.cpp:5-29).
#include "context.hpp"

using namespace pgrt;

namespace pgrt {

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
    // texel windows are addressed by 32-bit pool offsets (shade_ops.hpp tex_fetch)
    PGRT_REQUIRE(pool + 16 < (1ll << 32), PGRT_ERR_INVALID_ARGUMENT,
                 "textures of " + std::to_string(pool) + " bytes: the texel pool would exceed 4 GiB");
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
    // the traversal kernels address nodes and triangles by 32-bit byte offsets (common.hpp at_bytes,
    // the packet kernel's scalar loads): every array below 4 GiB -- up to ~53 M references
    PGRT_REQUIRE((unsigned long long)m * sizeof(Bvh8Node) < (1ull << 32), PGRT_ERR_INVALID_ARGUMENT,
                 "scene of " + std::to_string(m) + " triangle references: the BVH arrays would exceed 4 GiB");
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

}  // namespace pgrt
