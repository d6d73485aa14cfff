// camera_ops.hpp -- primary ray of a sample-batch slot, shared by k_raygen and the level-0 packet
// traversal (which generates the ray in registers and stores it for the level-0 shade, see
// DESIGN.md "fused primary rays").  Same float operation order in both, so the rays are
// bit-identical.
#pragma once

#include "cache_ops.hpp"

#include "shade_ops.hpp"
#include "trace.hpp"

namespace pgrt {

// slot pixel -> image pixel: 64x64 tiles, 8x8-pixel blocks inside (one wave = one block)
__device__ __forceinline__ void tile_pixel(int slot_pix, const int4* tiles, int& px, int& py, bool& valid) {
    const int tile = slot_pix / (kTile * kTile);
    const int p = slot_pix - tile * kTile * kTile;
    const int blk = p >> 6, w = p & 63;
    const int lx = ((blk & 7) << 3) + (w & 7);
    const int ly = ((blk >> 3) << 3) + (w >> 3);
    const int4 tr = tiles[tile];
    valid = lx < tile_width(tr) && ly < tr.w;
    px = tr.x + lx;
    py = tr.y + ly;
}

// Write the finished pixel o of batch slot pixel p (image pixel px, py) to fo.
__device__ __forceinline__ void store_pixel(const FrameParams& fp, const int4* tiles, const FrameOut& fo, int p,
                                            int px, int py, float4 o) {
    if (fo.mode == 0) {
        float* dst = fo.out + (size_t)frame_of_tile(tiles[p / (kTile * kTile)]) * fp.frame_stride +
                     ((size_t)(py - fo.oy) * (size_t)fo.pitch + (size_t)(px - fo.ox)) * 4;
        st_stream(reinterpret_cast<float4*>(dst), o);
        return;
    }
    const int tile = p / (kTile * kTile);
    const int4 tr = tiles[tile];
    size_t gtile = (size_t)tile * fo.K + fo.j;  // position in the caller's tile list
    if (fp.frame_tiles > 0) {  // multi-frame call: frame f's tiles start at f * frame_out_tiles
        const size_t f = gtile / fp.frame_tiles;
        gtile += f * (size_t)(fp.frame_out_tiles - fp.frame_tiles);
    }
    const size_t q = gtile * kTile * kTile + (size_t)(py - tr.y) * kTile + (size_t)(px - tr.x);
    if (fo.mode == 1) {
        st_stream(reinterpret_cast<float4*>(fo.out + q * 4), o);
    } else {  // 2: RGB only (alpha is always 1): the multi-GPU gather moves 12 B per pixel
        st_stream_nt(fo.out + q * 3 + 0, o.x);
        st_stream_nt(fo.out + q * 3 + 1, o.y);
        st_stream_nt(fo.out + q * 3 + 2, o.z);
    }
}

// Ray i of the batch (samples innermost): get_pixel's stratified sample position + jitter
// (APP/raytracer.cpp:396-416) through Camera::GenerateRay, pinhole (PinHoleCamera.cpp:31-63) or
// thin lens (:65-105).  ro = (org, tnear), rd = (dir, tfar).  Returns false for a padding slot
// of a partial tile: ro = 0, rd = (0, 0, 0, -1) (tfar < 0 never hits).
__device__ __forceinline__ bool primary_ray(const CameraView& cam, const FrameParams& fp, const int4* tiles, int i,
                                            float4& ro, float4& rd) {
    // one sample per pixel per batch (1 spp, the C2 frames): no integer divisions by run-time values
    const int slot_pix = fp.nsb == 1 ? i : i / fp.nsb;
    const int s = fp.s0 + (i - slot_pix * fp.nsb);
    int px, py;
    bool valid;
    tile_pixel(slot_pix, tiles, px, py, valid);
    if (!valid) {
        ro = make_float4(0, 0, 0, 0);
        rd = make_float4(0, 0, 0, -1.0f);
        return false;
    }
    const uint32_t frame = fp.frame + (uint32_t)frame_of_tile(tiles[slot_pix / (kTile * kTile)]);
    const int S = fp.spp_side;
    const int sq = S == 1 ? 0 : s / S;
    const int sx = sq, sy = s - sq * S;
    const uint32_t pixel = (uint32_t)py * (uint32_t)cam.width + (uint32_t)px;
    float j0 = 0.0f, j1 = 0.0f, j2 = 0.0f, j3 = 0.0f;
    if (fp.jitter != PGRT_JITTER_NONE) {
        const float ja = fp.jit_a, jb = fp.jit_b;  // -0.5f / S, 0.5f / S
        const float u0 = pg_jitter_u01(fp.seed, frame, pixel, (uint32_t)s, 0);
        const float u1 = pg_jitter_u01(fp.seed, frame, pixel, (uint32_t)s, 1);
        j0 = u0 * (jb - ja) + ja;
        j1 = u1 * (jb - ja) + ja;
        if (fp.dof) {  // the lens sample (streams 2, 3) only where the thin lens uses it
            const float la = -fp.aperture / 2.0f, lb = fp.aperture / 2.0f;
            const bool corr = fp.jitter == PGRT_JITTER_HASH_CORRELATED;
            const float u2 = corr ? u0 : pg_jitter_u01(fp.seed, frame, pixel, (uint32_t)s, 2);
            const float u3 = corr ? u1 : pg_jitter_u01(fp.seed, frame, pixel, (uint32_t)s, 3);
            j2 = u2 * (lb - la) + la;
            j3 = u3 * (lb - la) + la;
        }
    }
    // get_pixel sample position (raytracer.cpp:412-413)
    const float nx = (float)px + ((float)sx * fp.inv_s) + j0;  // fp.inv_s = 1.0f / S
    const float ny = (float)py + ((float)sy * fp.inv_s) + j1;
    // camera-space direction with integer W/2, H/2 (PinHoleCamera.cpp:41-42, :67)
    V3 crd = v3(nx - (float)(cam.width / 2), (float)(cam.height / 2) - ny, -cam.fy);
    crd = normalize(crd);
    V3 org, dir;
    float tnear;
    if (!fp.dof) {  // generate_ray(x, y) (PinHoleCamera.cpp:31-63)
        org = v3(cam.from[0], cam.from[1], cam.from[2]);
        dir = mat_mul(cam.m, crd);
        tnear = 0.001f;
    } else {  // generate_ray(x, y, focal, aperture) (PinHoleCamera.cpp:65-105)
        V3 dws = normalize(mat_mul(cam.m, crd));
        const V3 fpnt = v3(cam.from[0] + dws.x * fp.focal, cam.from[1] + dws.y * fp.focal,
                           cam.from[2] + dws.z * fp.focal);
        const V3 shift = mat_mul(cam.m, v3(j2, j3, 0));
        org = v3(cam.from[0] + shift.x, cam.from[1] + shift.y, cam.from[2] + shift.z);
        dir = normalize(v3(fpnt.x - org.x, fpnt.y - org.y, fpnt.z - org.z));
        tnear = 0.01f;
    }
    ro = make_float4(org.x, org.y, org.z, tnear);
    rd = make_float4(dir.x, dir.y, dir.z, 3.402823466e+38f);
    return true;
}

// level-0 rays regenerated in registers (no ray queue): the launch's camera, batch and tiles
struct PrimaryGen {
    CameraView cam;
    FrameParams fp;
    const int4* tiles;
    // the packet traversal stores the rays it generated (k_raygen's queue layout) for the
    // level-0 shade; pinhole frames store only the directions (store_ro = store_time = NULL:
    // every valid ray starts at the camera with tnear 0.001 in air, PinHoleCamera.cpp:31-63)
    float4* store_ro;
    float4* store_rd;
    float* store_time;
    int* store_count;  // the level-0 ray count (FrameCounters::count0), k_raygen's other output
    // 1-spp batches (L0Final): hit records are stored only for the rays that hit, and per wave
    // the mask of those lanes (NULL: a hit record for every ray)
    unsigned long long* hitmask;
};

// get_pixel's last step for batch slot pixel p of a 1-spp pixel whose sample colour is v:
// final_color = 0 + v (raytracer.cpp:422-429, the "+=" onto a zero colour is kept: -0 -> +0),
// gamma(Color4f{b, g, r}) (:431-435), written to fo (k_finish's output modes).
__device__ __forceinline__ void store_final_1spp(const FrameParams& fp, const int4* tiles, const FrameOut& fo, int p,
                                                 float4 v) {
    int px, py;
    bool valid;
    tile_pixel(p, tiles, px, py, valid);
    if (!valid) return;
    const float4 acc = make_float4(0.0f + v.x, 0.0f + v.y, 0.0f + v.z, 1.0f);
    store_pixel(fp, tiles, fo, p, px, py, gamma_rgba(acc.z, acc.y, acc.x, fp.gamma));
}

}  // namespace pgrt
