// shade_ops.hpp -- device restatement of the reference's per-hit arithmetic.
//
// Every function keeps the reference's float operation order (the library is compiled with
// -ffp-contract=off) so results are bit-identical to the CPU restatement in oracle/oracle.c.
// Reference anchors are given per function; src/pg/pg1_embree is abbreviated APP.
#pragma once

#include "common.hpp"

namespace pgrt {

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
// Vector3 operator*(float, Vector3) == operator*(Vector3, float) == a * v.c (APP/vector3.cpp:245-253)
__device__ __forceinline__ V3 scale(float a, V3 v) { return v3(a * v.x, a * v.y, a * v.z); }
// DotProduct (APP/vector3.cpp:187-190)
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// CrossProduct (APP/vector3.cpp:169-175)
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Normalize (APP/vector3.cpp:155-167)
__device__ __forceinline__ V3 normalize(V3 v) {
    const float norm = v.x * v.x + v.y * v.y + v.z * v.z;
    if (norm != 0) {
        const float rn = 1 / sqrtf(norm);
        v.x *= rn;
        v.y *= rn;
        v.z *= rn;
    }
    return v;
}
// L2Norm (APP/vector3.cpp:145-148)
__device__ __forceinline__ float length(V3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
// Matrix3x3 * Vector3 (APP/matrix3x3.cpp:68-73)
__device__ __forceinline__ V3 mat_mul(const float* m, V3 b) {
    return v3(m[0] * b.x + m[1] * b.y + m[2] * b.z, m[3] * b.x + m[4] * b.y + m[5] * b.z,
              m[6] * b.x + m[7] * b.y + m[8] * b.z);
}

// rtcInterpolate0 over de-indexed per-vertex attributes, Embree's madd(w,p0,madd(u,p1,v*p2))
__device__ __forceinline__ float interp1(float a0, float a1, float a2, float u, float v) {
    const float w = 1.0f - u - v;
    return fmaf(w, a0, fmaf(u, a1, v * a2));
}

// byte / 255.0f for every byte value, filled per block (k_shade) with the same correctly
// rounded division the reference performs per channel: a table read instead of a division
__device__ __forceinline__ void fill_byte_lut(float* lut) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lut[i] = (float)i / 255.0f;
    __syncthreads();
}

// Texture::get_pixel (APP/texture.cpp:56-62): Color3f{B,G,R}/255; bytes outside the decoded
// buffer read as 0 (the reference reads out of bounds there).  lut[b] == b / 255.0f.
__device__ __forceinline__ V3 tex_pixel(const DevTexture& t, const unsigned char* pool, const float* lut, int x,
                                        int y) {
    long long off = (long long)y * t.pitch + (long long)x * t.bpp;
    if (off < 0 || off + 2 >= t.size) return v3(0, 0, 0);
    const unsigned char* p = pool + t.offset + off;
    return v3(lut[p[0]], lut[p[1]], lut[p[2]]);
}

// Texture::get_texel (APP/texture.cpp:77-130): bilinear with the reference's edge quirks, in two
// halves so a kernel can issue a texel fetch, do other work (another ray's loads) and consume it
// later: tex_fetch computes the taps and issues the loads of the usual case, tex_finish waits for
// them and interpolates.  tex_texel == tex_finish(tex_fetch(...)).
struct TexTap {
    float x, y;
    int x1, x2, y1, y2;
    int mode;             // 0: black (edge quirk / non-finite); 1: row windows loaded; 2: edge taps
    unsigned w1[3], w2[3];  // the two rows' aligned 12-byte windows (mode 1)
    unsigned k1, k2;        // byte shift of each window
};
__device__ __forceinline__ TexTap tex_fetch(const DevTexture& t, const unsigned char* pool, float u, float v) {
    TexTap q;
    q.x = u * (float)t.width;
    q.y = v * (float)t.height;
    q.mode = 0;
    q.x1 = q.x2 = q.y1 = q.y2 = 0;
    q.k1 = q.k2 = 0;
    if (!(fabsf(q.x) < 16777216.0f) || !(fabsf(q.y) < 16777216.0f)) return q;
    const int tmp_x1 = (int)floorf(q.x), tmp_x2 = (int)ceilf(q.x);
    const int tmp_y1 = (int)floorf(q.y), tmp_y2 = (int)ceilf(q.y);
    q.x1 = (tmp_x1 < 1) ? tmp_x1 + 1 : tmp_x1;
    q.x2 = (tmp_x2 == t.width) ? 0 : tmp_x2;
    q.y1 = (tmp_y1 < 1) ? tmp_y1 + 1 : tmp_y1;
    q.y2 = (tmp_y2 == t.height) ? tmp_y1 : tmp_y2;
    if (q.x1 == q.x2 || q.y1 == q.y2) return q;
    const long long o1 = (long long)q.y1 * t.pitch + (long long)q.x1 * t.bpp;
    const long long o2 = (long long)q.y2 * t.pitch + (long long)q.x1 * t.bpp;
    if (q.x2 == q.x1 + 1 && t.bpp <= 4 && o1 >= 0 && o2 >= 0 && o1 + t.bpp + 2 < t.size && o2 + t.bpp + 2 < t.size) {
        // the usual case: both taps of a row are neighbours inside the texture -> one aligned
        // 12-byte window per row (the texel pool is padded for it) instead of 6 byte loads
        // 32-bit pool offsets (the pool stays below 4 GiB, set_scene checks; its base is 256-B
        // aligned, so an offset's low bits are the address's): a scalar base + one VGPR per load
        const unsigned f1 = (unsigned)t.offset + (unsigned)o1, f2 = (unsigned)t.offset + (unsigned)o2;
        q.k1 = f1 & 3u;
        q.k2 = f2 & 3u;
        const unsigned* a = at_bytes(reinterpret_cast<const unsigned*>(pool), f1 & ~3u);
        const unsigned* b = at_bytes(reinterpret_cast<const unsigned*>(pool), f2 & ~3u);
        q.w1[0] = a[0];
        q.w1[1] = a[1];
        q.w1[2] = a[2];
        q.w2[0] = b[0];
        q.w2[1] = b[1];
        q.w2[2] = b[2];
        q.mode = 1;
    } else {
        q.mode = 2;
    }
    return q;
}
// the two horizontally adjacent texels of a row window: bytes off .. off + 7 out of three aligned
// dwords by v_alignbyte_b32 funnel shifts (set_scene pads the texel pool for the 12-byte read)
__device__ __forceinline__ void tex_window_pair(int bpp, const float* lut, const unsigned* w, unsigned k, V3& a,
                                                V3& b) {
    const unsigned lo = __builtin_amdgcn_alignbyte(w[1], w[0], k);  // bytes off .. off + 3
    const unsigned hi = __builtin_amdgcn_alignbyte(w[2], w[1], k);  // bytes off + 4 .. off + 7
    a = v3(lut[lo & 0xffu], lut[(lo >> 8) & 0xffu], lut[(lo >> 16) & 0xffu]);
    if (bpp == 3)
        b = v3(lut[lo >> 24], lut[hi & 0xffu], lut[(hi >> 8) & 0xffu]);
    else
        b = v3(lut[hi & 0xffu], lut[(hi >> 8) & 0xffu], lut[(hi >> 16) & 0xffu]);
}
__device__ __forceinline__ V3 tex_finish(const TexTap& q, const DevTexture& t, const unsigned char* pool,
                                         const float* lut) {
    if (q.mode == 0) return v3(0, 0, 0);
    const float x = q.x, y = q.y;
    const int x1 = q.x1, x2 = q.x2, y1 = q.y1, y2 = q.y2;
    V3 x1y1, x2y1, x1y2, x2y2;
    if (q.mode == 1) {
        tex_window_pair(t.bpp, lut, q.w1, q.k1, x1y1, x2y1);
        tex_window_pair(t.bpp, lut, q.w2, q.k2, x1y2, x2y2);
    } else {
        x1y1 = tex_pixel(t, pool, lut, x1, y1);
        x2y1 = tex_pixel(t, pool, lut, x2, y1);
        x1y2 = tex_pixel(t, pool, lut, x1, y2);
        x2y2 = tex_pixel(t, pool, lut, x2, y2);
    }
    // the denominators are 1 except at the wrap / clamp quirks: q / 1 == q exactly, so the
    // (correctly rounded, ~10-instruction) division only runs where it can change the value
    const float dx = (float)(x2 - x1), dy = (float)(y2 - y1);
    const float Q11 = dx == 1.0f ? (float)x2 - x : ((float)x2 - x) / dx;
    const float Q21 = dx == 1.0f ? x - (float)x1 : (x - (float)x1) / dx;
    const float Q12 = Q11, Q22 = Q21;
    const V3 f1 = v3(x1y1.x * Q11 + x2y1.x * Q21, x1y1.y * Q11 + x2y1.y * Q21, x1y1.z * Q11 + x2y1.z * Q21);
    const V3 f2 = v3(x1y2.x * Q12 + x2y2.x * Q22, x1y2.y * Q12 + x2y2.y * Q22, x1y2.z * Q12 + x2y2.z * Q22);
    const float wy2 = dy == 1.0f ? (float)y2 - y : ((float)y2 - y) / dy;
    const float wy1 = dy == 1.0f ? y - (float)y1 : (y - (float)y1) / dy;
    return v3(f1.x * wy2 + f2.x * wy1, f1.y * wy2 + f2.y * wy1, f1.z * wy2 + f2.z * wy1);
}
__device__ inline V3 tex_texel(const DevTexture& t, const unsigned char* pool, const float* lut, float u, float v) {
    return tex_finish(tex_fetch(t, pool, u, v), t, pool, lut);
}

// ---- env-map angles, fast and still bit-identical to pg_atan2f / pg_asinf ----
// atan2 in double with FMA, a Newton-refined v_rcp_f64 instead of the correctly rounded divides,
// a 10-term series after the same pi/6 reduction (truncation < 5e-14 absolute) and a hardware
// sqrt for asin's cosine: within 1e-12 relative of the exact double pg_atan2_d computes (itself
// within 5e-15 of atan2).  Ziv's rounding test then decides: when a +- 1e-12 |a| rounds to ONE
// float, that float is (float)pg_atan2_d's result (rounding is monotonic); otherwise (about 3e-5
// of the lookups) the exact pgrt_detmath.h function runs.  Tested bit for bit against the
// exact functions on the device (pgrt_selftest_env, tests/test_gpu_parity.py).
__device__ __forceinline__ double rcp_refined(double d) {  // d normal and > 0: ~1 ulp
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    return fma(r, fma(-d, r, 1.0), r);
}
__device__ __forceinline__ double atan2_approx(double y, double x) {  // x, y finite, nonzero
    const double ay = fabs(y), ax = fabs(x);
    const bool swap = ay > ax;
    double q = (swap ? ax : ay) * rcp_refined(swap ? ay : ax);  // in (0, 1]
    double base = 0.0;
    if (q > 0.26794919243112270647) {  // tan(pi/12): atan q = pi/6 + atan((q sqrt3 - 1) / (q + sqrt3))
        q = fma(q, 1.73205080756887729353, -1.0) * rcp_refined(q + 1.73205080756887729353);
        base = PG_PI_D / 6.0;
    }
    const double z = q * q;  // <= 0.0718
    double p = -1.0 / 19.0;
    p = fma(p, z, 1.0 / 17.0);
    p = fma(p, z, -1.0 / 15.0);
    p = fma(p, z, 1.0 / 13.0);
    p = fma(p, z, -1.0 / 11.0);
    p = fma(p, z, 1.0 / 9.0);
    p = fma(p, z, -1.0 / 7.0);
    p = fma(p, z, 1.0 / 5.0);
    p = fma(p, z, -1.0 / 3.0);
    p = fma(p, z, 1.0);
    double r = fma(q, p, base);
    if (swap) r = PG_PI_D / 2.0 - r;
    if (x < 0.0) r = PG_PI_D - r;
    return y < 0.0 ? -r : r;
}
// (float)a's value when it is decided by a +- 1e-12 |a| (else NaN: undecided)
__device__ __forceinline__ float round_decided(double a) {
    const double e = fabs(a) * 1e-12;
    const float lo = (float)(a - e), hi = (float)(a + e);
    return lo == hi ? lo : __builtin_nanf("");
}
__device__ inline float atan2f_env(float y, float x) {  // == pg_atan2f(y, x)
    const float ay = fabsf(y), ax = fabsf(x);
    float f = __builtin_nanf("");
    if (ay > 1e-30f && ax > 1e-30f && ay < 1e30f && ax < 1e30f) f = round_decided(atan2_approx(y, x));
    return f == f ? f : pg_atan2f(y, x);
}
__device__ inline float asinf_env(float x) {  // == pg_asinf(x)
    float f = __builtin_nanf("");
    if (fabsf(x) > 1e-30f && fabsf(x) < 0.9999f) {
        const double xd = (double)x;
        f = round_decided(atan2_approx(xd, sqrt(1.0 - xd * xd)));
    }
    return f == f ? f : pg_asinf(x);
}

// SphericalMap::get_texel (APP/SphericalMap.cpp:17-29): returns RGBA with a = 1.  env_fetch /
// env_finish split it like tex_fetch / tex_finish (env_texel == env_finish(env_fetch(...))).
__device__ __forceinline__ TexTap env_fetch(const SceneView& s, V3 d) {
    if (s.env < 0) {
        TexTap q;
        q.mode = 0;
        return q;
    }
    const V3 vec = normalize(v3(d.x, d.z, d.y));
    // SphericalMap.cpp's divisions by 2 pi and pi as products with the double reciprocals: the
    // float results are identical for every float angle in [-pi, pi] / [-pi/2, pi/2] (exhaustive
    // check, tools/env_div_check.py; a double division is a ~10-instruction sequence)
    const float u = (float)(0.5 + (double)atan2f_env(vec.x, vec.z) * (1.0 / (2 * 3.14159265358979323846)));
    const float v = (float)(0.5 - (double)asinf_env(vec.y) * (1.0 / 3.14159265358979323846));
    return tex_fetch(s.tex[s.env], s.texels, u, v);
}
__device__ __forceinline__ float4 env_finish(const SceneView& s, const float* lut, const TexTap& q) {
    if (s.env < 0) return make_float4(0, 0, 0, 1);
    const V3 c = tex_finish(q, s.tex[s.env], s.texels, lut);
    return make_float4(c.z, c.y, c.x, 1.0f);
}
__device__ inline float4 env_texel(const SceneView& s, const float* lut, V3 d) {
    return env_finish(s, lut, env_fetch(s, d));
}

// utils.cpp:204-241, exactly as the restatement evaluates it (pg_pow_d: double exp(y log x))
__device__ __noinline__ float srgb_compress_exact(float u) {
    if (u <= 0) return 0.0f;
    if (u >= 1) return 1.0f;
    if ((double)u <= 0.00313080) return (float)(12.92 * (double)u);
    return (float)(1.00 * pg_pow_d((double)u, 1 / 2.4) - 0.055);
}
__device__ __noinline__ float srgb_expand_exact(float u) {
    if (u <= 0) return 0.0f;
    if (u >= 1) return 1.0f;
    if ((double)u <= 0.04045) return (float)((double)u / 12.92);
    return (float)pg_pow_d(((double)u + 0.055) / 1.055, 2.4);
}

// The same floats, faster (mix_srgb's six powers are most of a dielectric node's combine).  y =
// x^(p/q) as the root of y^q = x^p: a float exp2(log2) estimate (~2^-20 relative), then two Newton
// steps in double with a float reciprocal of the derivative (-> ~2^-50), then Ziv's rounding test:
// when y widened by 2^-40 either way rounds to one float, that float is also the rounding of the
// restatement's pg_pow_d (both are within ~2^-50 of the true power; the double exponents 2.4 and
// 1/2.4 differ from 12/5 and 5/12 by < 2^-51 relative in the result), otherwise the exact function
// decides (probability ~2^-16).  tests/test_gpu_parity.py compares both on EVERY float in [0, 1].
__device__ __forceinline__ double pow_root_newton(double y, double xp, int q) {
    // one Newton step for y^q = xp (q = 5 or 12): y -= (y^q - xp) / (q y^(q-1))
    const double y2 = y * y, y4 = y2 * y2;
    const double yq = q == 5 ? y4 * y : y4 * y4 * y4;
    const float r = __builtin_amdgcn_rcpf((float)((double)q * yq)) * (float)y;  // 1 / (q y^(q-1))
    return fma(-(yq - xp), (double)r, y);
}
__device__ inline float srgb_compress(float u) {
    if (u <= 0) return 0.0f;
    if (u >= 1) return 1.0f;
    if ((double)u <= 0.00313080) return (float)(12.92 * (double)u);
    const double x = (double)u;
    const double x2 = x * x, x5 = x2 * x2 * x;  // y = x^(5/12): y^12 = x^5
    double y = (double)__builtin_amdgcn_exp2f((5.0f / 12.0f) * __builtin_amdgcn_logf(u));
    y = pow_root_newton(y, x5, 12);
    y = pow_root_newton(y, x5, 12);
    const double v = y - 0.055, tol = y * 0x1p-40;
    const float lo = (float)(v - tol), hi = (float)(v + tol);
    return lo == hi ? lo : srgb_compress_exact(u);
}
__device__ inline float srgb_expand(float u) {
    if (u <= 0) return 0.0f;
    if (u >= 1) return 1.0f;
    if ((double)u <= 0.04045) return (float)((double)u / 12.92);
    const double x = ((double)u + 0.055) / 1.055;
    const double x4 = (x * x) * (x * x), x12 = x4 * x4 * x4;  // y = x^(12/5): y^5 = x^12
    double y = (double)__builtin_amdgcn_exp2f(2.4f * __builtin_amdgcn_logf((float)x));
    y = pow_root_newton(y, x12, 5);
    y = pow_root_newton(y, x12, 5);
    const double tol = y * 0x1p-40;
    const float lo = (float)(y - tol), hi = (float)(y + tol);
    return lo == hi ? lo : srgb_expand_exact(u);
}
// mix_srgb = compress(mix_linear(expand(c0), expand(c1), a)); each of the three swaps r<->b.
__device__ inline float4 mix_srgb(float4 c0, float4 c1, float a) {
    const float4 e0 = make_float4(srgb_expand(c0.z), srgb_expand(c0.y), srgb_expand(c0.x), 0.1f);
    const float4 e1 = make_float4(srgb_expand(c1.z), srgb_expand(c1.y), srgb_expand(c1.x), 0.1f);
    const float4 m = make_float4(a * e0.z + (1 - a) * e1.z, a * e0.y + (1 - a) * e1.y,
                                 a * e0.x + (1 - a) * e1.x, 1.0f);
    return make_float4(srgb_compress(m.z), srgb_compress(m.y), srgb_compress(m.x), 0.1f);
}

// pg_powf(x, g) with the gamma slider's default g = 0.5 (wave-uniform) decided once: pg_powf's
// y = 0.5 result is sqrtf(x) except at its earlier special cases that sqrtf does not share
// (+0 for x = -0, +inf for x = -inf); NaN / negative x give NaN either way
__device__ __forceinline__ float gamma_pow(float x, float g) {
    if (g == 0.5f) {
        if (x == 0.0f) return 0.0f;
        if (x == -__builtin_inff()) return __builtin_inff();
        return sqrtf(x);
    }
    return pg_powf(x, g);
}

// Raytracer::gamma (APP/raytracer.cpp:439-446) on Color4f{b,g,r} input: returns r,g,b order.
__device__ inline float4 gamma_rgba(float in_r, float in_g, float in_b, float g) {
    const float pb = gamma_pow(in_b, g), pg = gamma_pow(in_g, g), pr = gamma_pow(in_r, g);
    return make_float4(pb * pb, pg * pg, pr * pr, 1.0f);
}

// Ng = e2 x e1 of a triangle record (v0|id, e1, e2): the first step of tri_test, also
// precomputed per BVH reference (SceneView::tri_ng) with the same float operations
__host__ __device__ __forceinline__ float4 tri_normal(float4 q1, float4 q2) {
    const float e1x = q1.x, e1y = q1.y, e1z = q1.z;
    const float e2x = q2.x, e2y = q2.y, e2z = q2.z;
    return make_float4(e2y * e1z - e2z * e1y, e2z * e1x - e2x * e1z, e2x * e1y - e2y * e1x, 0.0f);
}

// Embree's Moeller-Trumbore triangle test (restated; see oracle.c tri_hit).
__device__ __forceinline__ float xorsign(float a, float s) {
    return __uint_as_float(__float_as_uint(a) ^ (__float_as_uint(s) & 0x80000000u));
}

}  // namespace pgrt
