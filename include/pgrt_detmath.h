/* pgrt_detmath.h -- deterministic scalar transcendentals shared by host and device.
 *
 * Why this exists: the reference (src/pg/pg1_embree, MSVC) calls the C/C++ math library for
 *   expf   -- dielectric attenuation          (raytracer.cpp:303-305, float overload of exp)
 *   powf   -- Phong specular, gamma           (raytracer.cpp:378-382, :441-443)
 *   pow    -- Fresnel-like R (double), sRGB   (raytracer.cpp:316, utils.cpp:208,215)
 *   atan2f/asinf -- spherical env map         (SphericalMap.cpp:22-23, float overloads
 *                                              from MSVC <cmath>, then double arithmetic)
 * Host libm (glibc) and the device math library (ocml) round these differently in the last
 * bit.  To make the GPU framebuffer bit-identical to the CPU restatement (oracle/), both sides
 * evaluate the functions below, written with IEEE-754 basic operations only (+ - * / and
 * conversions, no contraction -- the whole project builds with -ffp-contract=off), so every
 * result is the same bit pattern on x86-64 and gfx950.  Float functions are evaluated in
 * double and rounded once; their error against the correctly rounded result is < 1 ulp
 * (checked against glibc in tests/test_detmath.py).
 *
 * Usable from C (oracle), C++ (host) and HIP device code.
 */
#ifndef PGRT_DETMATH_H_
#define PGRT_DETMATH_H_

#include <stdint.h>
#if !defined(__HIPCC__) && !defined(__HIP__)
#include <math.h> /* sqrtf (IEEE correctly rounded on both targets) */
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#define PGRT_HD __host__ __device__ static inline
#else
#define PGRT_HD static inline
#endif

#define PG_PI_D 3.14159265358979323846
#define PG_INF_D (1.0 / 0.0)

PGRT_HD uint64_t pg_d2bits(double d) { union { double d; uint64_t u; } x; x.d = d; return x.u; }
PGRT_HD double pg_bits2d(uint64_t u) { union { double d; uint64_t u; } x; x.u = u; return x.d; }
PGRT_HD uint32_t pg_f2bits(float f) { union { float f; uint32_t u; } x; x.f = f; return x.u; }
PGRT_HD float pg_bits2f(uint32_t u) { union { float f; uint32_t u; } x; x.u = u; return x.f; }

PGRT_HD int pg_isnan_d(double x) { return x != x; }
PGRT_HD double pg_fabs_d(double x) { return pg_bits2d(pg_d2bits(x) & 0x7fffffffffffffffull); }
PGRT_HD float pg_fabsf(float x) { return pg_bits2f(pg_f2bits(x) & 0x7fffffffu); }

/* floor for |x| < 2^52 without libm: exact on both targets. */
PGRT_HD double pg_floor_d(double x)
{
    if (!(pg_fabs_d(x) < 4503599627370496.0)) return x; /* already integral, inf or nan */
    double t = (double)(int64_t)x;                       /* truncation toward zero (exact) */
    return (t > x) ? t - 1.0 : t;
}

/* 2^k as a double for -1022 <= k <= 1023 */
PGRT_HD double pg_pow2i(int k) { return pg_bits2d((uint64_t)(k + 1023) << 52); }

/* exp(x), relative error ~1e-16.  Cody-Waite reduction with fdlibm's split ln2. */
PGRT_HD double pg_exp(double x)
{
    if (x != x) return x;
    if (x > 709.782712893384) return PG_INF_D;
    if (x < -745.1332191019412) return 0.0;
    const double inv_ln2 = 1.44269504088896338700e+00;
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    double k = pg_floor_d(x * inv_ln2 + 0.5);
    double r = (x - k * ln2_hi) - k * ln2_lo; /* |r| <= ~0.3466 */
    /* Taylor to degree 13: truncation < 5e-18 relative */
    double p = 1.0 / 6227020800.0;           /* 1/13! */
    p = p * r + 1.0 / 479001600.0;           /* 1/12! */
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    int ki = (int)k;
    if (ki > 1023) return p * pg_pow2i(ki - 1) * 2.0;
    if (ki < -1021) return (p * pg_pow2i(ki + 600)) * pg_pow2i(-600);
    return p * pg_pow2i(ki);
}

/* natural log for finite x > 0 (callers handle the special cases). */
PGRT_HD double pg_log_pos(double x)
{
    int e = 0;
    if (x < 2.2250738585072014e-308) { x *= 18014398509481984.0; e = -54; } /* 2^54 */
    uint64_t b = pg_d2bits(x);
    e += (int)((b >> 52) & 0x7ff) - 1023;
    double m = pg_bits2d((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull); /* [1,2) */
    if (m > 1.41421356237309504880) { m = m * 0.5; e += 1; }                  /* (0.707,1.414] */
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    double s = (m - 1.0) / (m + 1.0); /* |s| <= 0.1716 */
    double z = s * s;
    double p = 1.0 / 25.0;
    p = p * z + 1.0 / 23.0;
    p = p * z + 1.0 / 21.0;
    p = p * z + 1.0 / 19.0;
    p = p * z + 1.0 / 17.0;
    p = p * z + 1.0 / 15.0;
    p = p * z + 1.0 / 13.0;
    p = p * z + 1.0 / 11.0;
    p = p * z + 1.0 / 9.0;
    p = p * z + 1.0 / 7.0;
    p = p * z + 1.0 / 5.0;
    p = p * z + 1.0 / 3.0;
    double lm = 2.0 * s + (2.0 * s) * (z * p); /* log(m) = 2 atanh(s) */
    double ed = (double)e;
    return ed * ln2_hi + (ed * ln2_lo + lm);
}

/* pow for finite x > 0 (used by the sRGB companding of utils.cpp:204-215). */
PGRT_HD double pg_pow_pos(double x, double y)
{
    if (x == 1.0) return 1.0;
    return pg_exp(y * pg_log_pos(x));
}

/* x^n for 0 < n <= 64 by squaring (each product rounded once, IEEE double) */
PGRT_HD double pg_ipow_d(double x, int n)
{
    double acc = 1.0;
    while (n) {
        if (n & 1) acc *= x;
        n >>= 1;
        if (n) x *= x;
    }
    return acc;
}

/* pow(double, double) for finite arguments with an integer or positive-base case split
 * (the Fresnel-like R of raytracer.cpp:316 raises 1 - |cos| to the 5th power in double). */
PGRT_HD double pg_pow_d(double x, double y)
{
    if (y == 0.0 || x == 1.0) return 1.0;
    if (x != x || y != y) return x + y;
    if (x > 0.0 && y >= 1.0 && y <= 64.0 && pg_floor_d(y) == y) return pg_ipow_d(x, (int)y); /* (1-cos)^5 */
    if (x > 0.0) return pg_exp(y * pg_log_pos(x));
    double fy = pg_floor_d(y);
    int odd = (fy == y) && (pg_fabs_d(y) < 9007199254740992.0) &&
              (((int64_t)fy) & 1);
    if (x == 0.0) {
        double r = (y > 0.0) ? 0.0 : PG_INF_D;
        return ((pg_d2bits(x) >> 63) && odd) ? -r : r;
    }
    if (fy != y) return (x - x) / (x - x);
    double r = pg_exp(y * pg_log_pos(-x));
    return odd ? -r : r;
}

PGRT_HD int pg_is_int_f(float y) /* 0 = not integer, 1 = even integer, 2 = odd integer */
{
    float ay = pg_fabsf(y);
    if (!(ay < 16777216.0f)) return (ay == ay && ay != PG_INF_D) ? 1 : 0; /* huge: even */
    int64_t i = (int64_t)ay;
    if ((float)i != ay) return 0;
    return (i & 1) ? 2 : 1;
}

/* powf with C99 Annex F special cases; general case via double exp(y*log|x|). */
PGRT_HD float pg_powf(float x, float y)
{
    if (y == 0.0f) return 1.0f;
    if (x == 1.0f) return 1.0f;
    if (x != x || y != y) return x + y;
    float ax = pg_fabsf(x), ay = pg_fabsf(y);
    int yint = pg_is_int_f(y);
    int neg = (pg_f2bits(x) >> 31) != 0;
    const float inf = (float)PG_INF_D;
    if (ay == inf) {
        if (ax == 1.0f) return 1.0f; /* (-1)^inf */
        int big = ax > 1.0f;
        return ((y > 0) == big) ? inf : 0.0f;
    }
    if (ax == inf) {
        float r = (y > 0) ? inf : 0.0f;
        return (neg && yint == 2) ? -r : r;
    }
    if (ax == 0.0f) {
        float r = (y > 0) ? 0.0f : inf;
        return (neg && yint == 2) ? -r : r;
    }
    if (neg && yint == 0) return (x - x) / (x - x); /* NaN: negative base, non-integer exponent */
    /* y = 1/2 (the gamma slider default): the correctly rounded sqrtf, identical on both
     * targets; exp(log/2) in double misrounds 48 of the 2^31 positive floats (checked) */
    if (y == 0.5f) return sqrtf(x);
    if (yint != 0 && ay <= 64.0f) {
        /* small integer exponent (Phong's Ns, raytracer.cpp:374-382): exponentiation by
         * squaring in double, <= 63 roundings of 2^-53 -> within 1 ulp after the final rounding,
         * and ~20x cheaper than exp(y log x) in double on both targets */
        double r = pg_ipow_d((double)ax, (int)ay);
        if (y < 0) r = 1.0 / r;
        float rf = (float)r;
        return (neg && yint == 2) ? -rf : rf;
    }
    double r = pg_exp((double)y * pg_log_pos((double)ax));
    float rf = (float)r;
    return (neg && yint == 2) ? -rf : rf;
}

PGRT_HD float pg_expf(float x) { return (float)pg_exp((double)x); }

/* atan for |a| in [0,1]: reduction around pi/6, then the Taylor series. */
PGRT_HD double pg_atan_01(double a)
{
    const double tan_pi_12 = 0.26794919243112270647;
    const double sqrt3 = 1.73205080756887729353;
    double base = 0.0;
    if (a > tan_pi_12) {
        a = (a * sqrt3 - 1.0) / (a + sqrt3);
        base = PG_PI_D / 6.0;
    }
    double z = a * a; /* <= 0.0718 */
    double p = -1.0 / 31.0;
    p = p * z + 1.0 / 29.0;
    p = p * z - 1.0 / 27.0;
    p = p * z + 1.0 / 25.0;
    p = p * z - 1.0 / 23.0;
    p = p * z + 1.0 / 21.0;
    p = p * z - 1.0 / 19.0;
    p = p * z + 1.0 / 17.0;
    p = p * z - 1.0 / 15.0;
    p = p * z + 1.0 / 13.0;
    p = p * z - 1.0 / 11.0;
    p = p * z + 1.0 / 9.0;
    p = p * z - 1.0 / 7.0;
    p = p * z + 1.0 / 5.0;
    p = p * z - 1.0 / 3.0;
    return base + (a + a * (z * p));
}

PGRT_HD double pg_atan_d(double x)
{
    if (x != x) return x;
    double a = pg_fabs_d(x);
    double r;
    if (a > 1.0) r = (a == PG_INF_D) ? PG_PI_D / 2.0 : PG_PI_D / 2.0 - pg_atan_01(1.0 / a);
    else r = pg_atan_01(a);
    return (x < 0) ? -r : r;
}

/* atan2 with the C99 special cases for zeros and infinities. */
PGRT_HD double pg_atan2_d(double y, double x)
{
    if (x != x || y != y) return x + y;
    int ys = (pg_d2bits(y) >> 63) != 0, xs = (pg_d2bits(x) >> 63) != 0;
    double ay = pg_fabs_d(y), ax = pg_fabs_d(x);
    double r;
    if (ay == 0.0) {
        r = xs ? PG_PI_D : 0.0;
    } else if (ax == 0.0) {
        r = PG_PI_D / 2.0;
    } else if (ax == PG_INF_D) {
        if (ay == PG_INF_D) r = xs ? 3.0 * PG_PI_D / 4.0 : PG_PI_D / 4.0;
        else r = xs ? PG_PI_D : 0.0;
    } else if (ay == PG_INF_D) {
        r = PG_PI_D / 2.0;
    } else {
        double t = pg_atan_d(ay / ax);
        r = xs ? PG_PI_D - t : t;
    }
    return ys ? -r : r;
}

/* sqrt of a normal double > 0 by Newton iteration from an exponent-halved guess: basic ops
 * only, so host and device agree bit for bit (the guess is within a factor 1.5 of the root,
 * six steps reach full double precision). */
PGRT_HD double pg_sqrt_d(double d)
{
    if (!(d > 0.0)) return (d == 0.0) ? d : (d - d) / (d - d);
    uint64_t b = pg_d2bits(d);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    int h = (e >= 0) ? e / 2 : -((1 - e) / 2); /* floor(e/2) */
    double g = pg_pow2i(h) * ((e - 2 * h) ? 1.4 : 1.0);
    for (int i = 0; i < 6; ++i) g = 0.5 * (g + d / g);
    return g;
}

PGRT_HD float pg_atan2f(float y, float x) { return (float)pg_atan2_d((double)y, (double)x); }

PGRT_HD float pg_asinf(float x)
{
    if (x != x) return x;
    if (pg_fabsf(x) > 1.0f) return (x - x) / (x - x);
    double xd = (double)x;
    double c = 1.0 - xd * xd; /* exact: x has 24 significant bits */
    return (float)pg_atan2_d(xd, pg_sqrt_d(c));
}

/* ---- deterministic sample jitter (replaces the wall-clock seeded std::mt19937 of
 *      raytracer.cpp:407-410 and PinHoleCamera.cpp:120-123) ----
 * u = U[0,1) from a counter hash of (seed, frame, global pixel index, sample, stream);
 * streams: 0,1 = pixel jitter r1,r2; 2,3 = lens offsets.  Values scale like
 * std::uniform_real_distribution: u * (b - a) + a. */
PGRT_HD uint32_t pg_hash32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

PGRT_HD float pg_jitter_u01(uint32_t seed, uint32_t frame, uint32_t pixel, uint32_t sample,
                            uint32_t stream)
{
    uint32_t h = pg_hash32(pg_hash32(pg_hash32(pg_hash32(seed) ^ frame) ^ pixel) ^
                           (sample * 4u + stream));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

/* ---- path tracing random numbers (PGRT_MODE_PATH) ----
 * key = counter hash of (seed, frame, global pixel, sample) -- a stream of its own, apart from
 * pg_jitter_u01's; u = U[0,1) for (bounce, k) of that path: k = 0 the dielectric choice,
 * k = 1 + 2j, 2 + 2j the j-th disk-sample candidate of a diffuse bounce. */
PGRT_HD uint32_t pg_path_key(uint32_t seed, uint32_t frame, uint32_t pixel, uint32_t sample)
{
    return pg_hash32(pg_hash32(pg_hash32(pg_hash32(seed ^ 0x68bc21ebu) ^ frame) ^ pixel) ^ sample);
}

PGRT_HD float pg_path_u01(uint32_t key, uint32_t bounce, uint32_t k)
{
    uint32_t h = pg_hash32(key ^ pg_hash32(bounce * 64u + k + 1u));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

#endif /* PGRT_DETMATH_H_ */
