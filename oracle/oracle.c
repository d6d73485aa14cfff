/* oracle.c -- CPU restatement of the reference Whitted trace path (TEST INFRASTRUCTURE).
 *
 * Restates, function by function, src/pg/pg1_embree of rddrdhd/PGI_RayTracing:
 *   PinHoleCamera (PinHoleCamera.cpp:5-105), Raytracer::get_pixel/trace/is_illuminated/
 *   get_reflection_ray/get_refraction_ray/gamma (raytracer.cpp:150-446), Texture::get_texel/
 *   get_pixel (texture.cpp:56-130), SphericalMap::get_texel (SphericalMap.cpp:17-29),
 *   LightSource::GenerateRay (LightSource.cpp:11-32), mix_srgb & co (utils.cpp:204-241),
 *   Vector3/Matrix3x3 arithmetic (vector3.cpp, matrix3x3.cpp:32-73).
 * Embree 3.11 (absent binary, headers only) is restated as: closest hit in (tnear, tfar]
 * (rtcIntersect1, embree doc README.md:6354-6394), the Moeller-Trumbore form of Embree's
 * triangle intersector (e1 = v0-v1, e2 = v2-v0, Ng = e2 x e1; edge tests on the scaled
 * U,V before the division), and rtcInterpolate's madd(w,p0,madd(u,p1,v*p2)) with
 * w = 1-u-v (rtcore_geometry.h:288-305).  Ties in t go to the smaller global triangle index.
 *
 * Float semantics follow the MSVC build of the reference: float overloads of sqrt/exp/pow/
 * atan2/asin/abs (MSVC <cmath> puts them in the global namespace), double pow for
 * pow(float,int) and pow(float,double).  Built with -ffp-contract=off.  Transcendentals
 * come from include/pgrt_detmath.h (bit-identical on host and device); -DORACLE_LIBM swaps
 * in glibc's for the cross-check in tests/test_oracle.py.
 */
#include "oracle.h"
#include "pgrt_detmath.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifdef ORACLE_LIBM
#define M_EXPF(x) expf(x)
#define M_POWF(x, y) powf(x, y)
#define M_POWD(x, y) pow(x, y)
#define M_ATAN2F(y, x) atan2f(y, x)
#define M_ASINF(x) asinf(x)
#else
#define M_EXPF(x) pg_expf(x)
#define M_POWF(x, y) pg_powf(x, y)
#define M_POWD(x, y) pg_pow_d(x, y)
#define M_ATAN2F(y, x) pg_atan2f(y, x)
#define M_ASINF(x) pg_asinf(x)
#endif

int orc_uses_libm(void)
{
#ifdef ORACLE_LIBM
    return 1;
#else
    return 0;
#endif
}

/* ------------------------------------------------------------------ vector3.cpp */
typedef struct { float x, y, z; } V3;
typedef struct { float r, g, b, a; } C4; /* Color4f (structs.h:11-14) */
typedef struct { float r, g, b; } C3;    /* Color3f (structs.h:16) */

static inline V3 v3(float x, float y, float z) { V3 v = {x, y, z}; return v; }
static inline V3 v_add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 v_sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 v_neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
/* operator*(float a, Vector3 v) and operator*(Vector3 v, float a) both form a*v.c (:245-253) */
static inline V3 v_scale(float a, V3 v) { return v3(a * v.x, a * v.y, a * v.z); }
/* DotProduct (vector3.cpp:187-190) */
static inline float v_dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* CrossProduct (vector3.cpp:169-175) */
static inline V3 v_cross(V3 a, V3 b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* Normalize (vector3.cpp:155-167): rn = 1/sqrt(|v|^2) in float, skipped for a zero vector */
static inline V3 v_normalize(V3 v)
{
    const float norm = v.x * v.x + v.y * v.y + v.z * v.z;
    if (norm != 0) {
        const float rn = 1 / sqrtf(norm);
        v.x *= rn;
        v.y *= rn;
        v.z *= rn;
    }
    return v;
}
/* L2Norm (vector3.cpp:145-148) */
static inline float v_len(V3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }

/* ------------------------------------------------------------------ PinHoleCamera */
typedef struct {
    int width, height;
    float f_y;
    V3 from;
    float m[9]; /* Matrix3x3 row-major; columns are x_c, y_c, z_c (matrix3x3.cpp:32-45) */
} Cam;

/* operator*(Matrix3x3, Vector3) (matrix3x3.cpp:68-73) */
static inline V3 m_mul(const float* m, V3 b)
{
    return v3(m[0] * b.x + m[1] * b.y + m[2] * b.z, m[3] * b.x + m[4] * b.y + m[5] * b.z,
              m[6] * b.x + m[7] * b.y + m[8] * b.z);
}

/* PinHoleCamera::PinHoleCamera (PinHoleCamera.cpp:5-29) */
static Cam cam_make(const pgrt_camera* c)
{
    Cam k;
    k.width = c->width;
    k.height = c->height;
    k.f_y = (float)c->height / (2 * tanf(c->fov_y / 2));
    k.from = v3(c->from[0], c->from[1], c->from[2]);
    V3 at = v3(c->at[0], c->at[1], c->at[2]);
    V3 up = v3(c->up[0], c->up[1], c->up[2]);
    V3 z_c = v_sub(k.from, at);
    V3 x_c = v_cross(up, z_c);
    V3 y_c = v_cross(z_c, x_c);
    z_c = v_normalize(z_c);
    x_c = v_normalize(x_c);
    y_c = v_normalize(y_c);
    k.m[0] = x_c.x; k.m[1] = y_c.x; k.m[2] = z_c.x;
    k.m[3] = x_c.y; k.m[4] = y_c.y; k.m[5] = z_c.y;
    k.m[6] = x_c.z; k.m[7] = y_c.z; k.m[8] = z_c.z;
    return k;
}

typedef struct {
    V3 org, dir;
    float tnear, tfar, time;
} Ray;

/* PinHoleCamera::generate_ray(x, y) (PinHoleCamera.cpp:31-63); W/2, H/2 are int divisions */
static Ray cam_ray_pinhole(const Cam* k, float x_i, float y_i)
{
    Ray r;
    r.org = k->from;
    V3 d = v3(x_i - (float)(k->width / 2), (float)(k->height / 2) - y_i, -k->f_y);
    d = v_normalize(d);
    r.dir = m_mul(k->m, d);
    r.tnear = 0.001f;
    r.tfar = FLT_MAX;
    r.time = 0.0f;
    return r;
}

/* PinHoleCamera::generate_ray(x, y, focal, aperture) (PinHoleCamera.cpp:65-105); the square
 * lens offset (rand1, rand2) ~ U(-a/2, a/2)^2 is passed in. */
static Ray cam_ray_dof(const Cam* k, float x_i, float y_i, float focal, float rand1,
                       float rand2)
{
    V3 crd = v3(x_i - (float)(k->width / 2), (float)(k->height / 2) - y_i, -k->f_y);
    crd = v_normalize(crd);
    V3 dws = m_mul(k->m, crd);
    dws = v_normalize(dws);
    V3 fp = v3(k->from.x + dws.x * focal, k->from.y + dws.y * focal, k->from.z + dws.z * focal);
    V3 shift = m_mul(k->m, v3(rand1, rand2, 0));
    Ray r;
    r.org = v3(k->from.x + shift.x, k->from.y + shift.y, k->from.z + shift.z);
    V3 nd = v3(fp.x - r.org.x, fp.y - r.org.y, fp.z - r.org.z);
    r.dir = v_normalize(nd);
    r.tnear = 0.01f;
    r.tfar = FLT_MAX;
    r.time = 0.0f;
    return r;
}

/* ------------------------------------------------------------------ scene + BVH */
typedef struct {
    float lo[3], hi[3];
    int left, right; /* internal: children; leaf: left = -1, right = first, cnt = count */
    int cnt;
} BNode;

struct orc_scene {
    int ntri;
    float* pos;  /* 9N */
    float* nrm;  /* 9N */
    float* uv;   /* 6N */
    int* mat;    /* N */
    float* pre;  /* 12N: v0, e1, e2, Ng */
    int nmat;
    pgrt_material* mats;
    int ntex;
    pgrt_texture* tex;
    unsigned char** texdata;
    int env;
    int nlight;
    pgrt_light* lights;
    int accel;
    BNode* nodes;
    int nnodes;
    int* perm;
    float pad;
};

static void tri_precompute(orc_scene* s)
{
    for (int i = 0; i < s->ntri; ++i) {
        const float* p = s->pos + 9 * i;
        V3 v0 = v3(p[0], p[1], p[2]), v1 = v3(p[3], p[4], p[5]), v2 = v3(p[6], p[7], p[8]);
        V3 e1 = v_sub(v0, v1), e2 = v_sub(v2, v0);
        V3 ng = v_cross(e2, e1);
        float* q = s->pre + 12 * i;
        q[0] = v0.x; q[1] = v0.y; q[2] = v0.z;
        q[3] = e1.x; q[4] = e1.y; q[5] = e1.z;
        q[6] = e2.x; q[7] = e2.y; q[8] = e2.z;
        q[9] = ng.x; q[10] = ng.y; q[11] = ng.z;
    }
}

static inline float xorsign(float a, float s_signbit_src)
{
    uint32_t ua, us;
    memcpy(&ua, &a, 4);
    memcpy(&us, &s_signbit_src, 4);
    ua ^= (us & 0x80000000u);
    memcpy(&a, &ua, 4);
    return a;
}

/* Embree's Moeller-Trumbore triangle test (restated; Embree 3.11 kernels/geometry/
 * triangle_intersector_moeller.h, not vendored): edge tests on the scaled U, V, then the depth
 * test on the SCALED distance, absDen*tnear < T <= absDen*tfar, and only then t = T / absDen
 * (Embree: T * rcp(absDen); here the IEEE division -- the one remaining difference).  The
 * interval is the ray's own (tnear, tfar], so the accepted set does not depend on the order in
 * which triangles are tested; the closest of them wins, ties to the smaller index. */
static inline int tri_hit(const float* q, const Ray* r, float* tt, float* uu, float* vv)
{
    V3 v0 = v3(q[0], q[1], q[2]), e1 = v3(q[3], q[4], q[5]), e2 = v3(q[6], q[7], q[8]);
    V3 ng = v3(q[9], q[10], q[11]);
    V3 C = v_sub(v0, r->org);
    V3 R = v_cross(C, r->dir);
    float den = v_dot(ng, r->dir);
    float absden = fabsf(den);
    float U = xorsign(v_dot(R, e2), den);
    float V = xorsign(v_dot(R, e1), den);
    if (!(den != 0.0f && U >= 0.0f && V >= 0.0f && U + V <= absden)) return 0;
    float T = xorsign(v_dot(ng, C), den);
    if (!(absden * r->tnear < T && T <= absden * r->tfar)) return 0;
    *tt = T / absden;
    *uu = U / absden;
    *vv = V / absden;
    return 1;
}

typedef struct {
    float t, u, v;
    int prim;
} Hit;

static inline void hit_consider(Hit* h, int prim, float t, float u, float v)
{
    if (h->prim < 0 || t < h->t || (t == h->t && prim < h->prim)) {
        h->t = t;
        h->u = u;
        h->v = v;
        h->prim = prim;
    }
}

/* ---- binned SAH BVH (the oracle's own acceleration structure; results do not depend on
 *      it because box culling is conservative and hits are tie-broken by index) ---- */
typedef struct {
    float lo[3], hi[3];
} Box;

static inline void box_empty(Box* b)
{
    for (int k = 0; k < 3; ++k) { b->lo[k] = FLT_MAX; b->hi[k] = -FLT_MAX; }
}
static inline void box_grow(Box* b, const Box* o)
{
    for (int k = 0; k < 3; ++k) {
        if (o->lo[k] < b->lo[k]) b->lo[k] = o->lo[k];
        if (o->hi[k] > b->hi[k]) b->hi[k] = o->hi[k];
    }
}
static inline float box_area(const Box* b)
{
    float dx = b->hi[0] - b->lo[0], dy = b->hi[1] - b->lo[1], dz = b->hi[2] - b->lo[2];
    if (dx < 0) return 0;
    return 2 * (dx * dy + dy * dz + dz * dx);
}

typedef struct {
    Box* tb;
    float* cen;
    int* perm;
    BNode* nodes;
    int nn;
    int cap;
} Build;

static int build_rec(Build* B, int first, int count, int depth)
{
    int ni = B->nn++;
    BNode* n = &B->nodes[ni];
    Box bb, cb;
    box_empty(&bb);
    box_empty(&cb);
    for (int i = first; i < first + count; ++i) {
        int t = B->perm[i];
        box_grow(&bb, &B->tb[t]);
        Box c;
        for (int k = 0; k < 3; ++k) c.lo[k] = c.hi[k] = B->cen[3 * t + k];
        box_grow(&cb, &c);
    }
    for (int k = 0; k < 3; ++k) { n->lo[k] = bb.lo[k]; n->hi[k] = bb.hi[k]; }
    if (count <= 4 || depth > 60) {
        n->left = -1; n->right = first; n->cnt = count;
        return ni;
    }
    enum { NB = 16 };
    float best_cost = FLT_MAX;
    int best_axis = -1, best_split = 0;
    for (int ax = 0; ax < 3; ++ax) {
        float ext = cb.hi[ax] - cb.lo[ax];
        if (!(ext > 0)) continue;
        Box bin[NB];
        int bc[NB];
        for (int b = 0; b < NB; ++b) { box_empty(&bin[b]); bc[b] = 0; }
        for (int i = first; i < first + count; ++i) {
            int t = B->perm[i];
            int b = (int)((B->cen[3 * t + ax] - cb.lo[ax]) / ext * NB);
            if (b >= NB) b = NB - 1;
            if (b < 0) b = 0;
            bc[b]++;
            box_grow(&bin[b], &B->tb[t]);
        }
        float lA[NB];
        int lC[NB];
        Box acc;
        box_empty(&acc);
        int c = 0;
        for (int b = 0; b < NB; ++b) { box_grow(&acc, &bin[b]); c += bc[b]; lA[b] = box_area(&acc); lC[b] = c; }
        box_empty(&acc);
        c = 0;
        for (int b = NB - 1; b > 0; --b) {
            box_grow(&acc, &bin[b]);
            c += bc[b];
            float cost = lA[b - 1] * lC[b - 1] + box_area(&acc) * c;
            if (lC[b - 1] > 0 && c > 0 && cost < best_cost) {
                best_cost = cost; best_axis = ax; best_split = b;
            }
        }
    }
    int mid;
    if (best_axis < 0) {
        mid = first + count / 2;
    } else {
        float ext = cb.hi[best_axis] - cb.lo[best_axis];
        int i = first, j = first + count - 1;
        while (i <= j) {
            int t = B->perm[i];
            int b = (int)((B->cen[3 * t + best_axis] - cb.lo[best_axis]) / ext * NB);
            if (b >= NB) b = NB - 1;
            if (b < 0) b = 0;
            if (b < best_split) ++i;
            else { int tmp = B->perm[i]; B->perm[i] = B->perm[j]; B->perm[j] = tmp; --j; }
        }
        mid = i;
        if (mid == first || mid == first + count) mid = first + count / 2;
    }
    int l = build_rec(B, first, mid - first, depth + 1);
    int r = build_rec(B, mid, first + count - mid, depth + 1);
    n = &B->nodes[ni];
    n->left = l; n->right = r; n->cnt = 0;
    return ni;
}

static void bvh_build(orc_scene* s)
{
    int N = s->ntri;
    Build B;
    B.tb = (Box*)malloc(sizeof(Box) * (size_t)(N > 0 ? N : 1));
    B.cen = (float*)malloc(sizeof(float) * 3 * (size_t)(N > 0 ? N : 1));
    B.perm = (int*)malloc(sizeof(int) * (size_t)(N > 0 ? N : 1));
    B.cap = 2 * N + 1;
    B.nodes = (BNode*)malloc(sizeof(BNode) * (size_t)B.cap);
    B.nn = 0;
    float glo = FLT_MAX, ghi = -FLT_MAX;
    for (int i = 0; i < N; ++i) {
        const float* p = s->pos + 9 * i;
        Box b;
        box_empty(&b);
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) {
                float c = p[3 * v + k];
                if (c < b.lo[k]) b.lo[k] = c;
                if (c > b.hi[k]) b.hi[k] = c;
                if (c < glo) glo = c;
                if (c > ghi) ghi = c;
            }
        B.tb[i] = b;
        for (int k = 0; k < 3; ++k) B.cen[3 * i + k] = 0.5f * (b.lo[k] + b.hi[k]);
        B.perm[i] = i;
    }
    /* conservative padding (world units) so rounding in the slab test never culls a box that
     * holds a triangle the triangle test accepts */
    s->pad = (N > 0) ? 1e-5f * (ghi - glo) + 1e-30f : 0.0f;
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 3; ++k) { B.tb[i].lo[k] -= s->pad; B.tb[i].hi[k] += s->pad; }
    if (N > 0) build_rec(&B, 0, N, 0);
    s->nodes = B.nodes;
    s->nnodes = B.nn;
    s->perm = B.perm;
    free(B.tb);
    free(B.cen);
}

static inline int slab(const BNode* n, const float* o, const float* id, float tmax, float* tent)
{
    float t0 = 0.0f, t1 = tmax;
    for (int k = 0; k < 3; ++k) {
        float a = (n->lo[k] - o[k]) * id[k];
        float b = (n->hi[k] - o[k]) * id[k];
        float lo = a < b ? a : b, hi = a < b ? b : a;
        if (lo > t0) t0 = lo;
        if (hi < t1) t1 = hi;
    }
    *tent = t0;
    return t0 <= t1 * 1.000001f;
}

/* rtcIntersect1: closest hit in (tnear, tfar] */
static Hit scene_intersect(const orc_scene* s, const Ray* r, uint64_t* tests)
{
    Hit h;
    h.prim = -1;
    h.t = r->tfar;
    h.u = h.v = 0.0f;
    float t, u, v;
    if (!s->accel) {
        for (int i = 0; i < s->ntri; ++i)
            if (tri_hit(s->pre + 12 * i, r, &t, &u, &v)) hit_consider(&h, i, t, u, v);
        if (tests) *tests += (uint64_t)s->ntri;
        return h;
    }
    if (s->nnodes == 0) return h;
    float o[3] = {r->org.x, r->org.y, r->org.z};
    float d[3] = {r->dir.x, r->dir.y, r->dir.z};
    float id[3];
    for (int k = 0; k < 3; ++k) {
        float dk = d[k];
        if (fabsf(dk) < 1e-30f) dk = (dk < 0 || (dk == 0 && signbit(dk))) ? -1e-30f : 1e-30f;
        id[k] = 1.0f / dk;
    }
    int stack[128];
    int sp = 0;
    float te;
    if (!slab(&s->nodes[0], o, id, FLT_MAX, &te)) return h;
    stack[sp++] = 0;
    while (sp > 0) {
        const BNode* n = &s->nodes[stack[--sp]];
        float tcur = (h.prim >= 0) ? h.t : r->tfar;
        if (n->left < 0) {
            for (int i = n->right; i < n->right + n->cnt; ++i) {
                int tri = s->perm[i];
                if (tests) ++*tests;
                if (tri_hit(s->pre + 12 * tri, r, &t, &u, &v)) hit_consider(&h, tri, t, u, v);
            }
            continue;
        }
        if (tests) ++tests[1]; /* node visits (tests[1] is Counters.visits) */
        float ta, tb;
        int ha = slab(&s->nodes[n->left], o, id, tcur, &ta);
        int hb = slab(&s->nodes[n->right], o, id, tcur, &tb);
        if (ha && hb) {
            if (ta <= tb) { stack[sp++] = n->right; stack[sp++] = n->left; }
            else { stack[sp++] = n->left; stack[sp++] = n->right; }
        } else if (ha) {
            stack[sp++] = n->left;
        } else if (hb) {
            stack[sp++] = n->right;
        }
    }
    return h;
}

/* rtcInterpolate0 over de-indexed per-vertex attributes: madd(w,p0,madd(u,p1,v*p2)) */
static inline float interp1(float a0, float a1, float a2, float u, float v)
{
    const float w = 1.0f - u - v;
    return fmaf(w, a0, fmaf(u, a1, v * a2));
}

/* ------------------------------------------------------------------ texture.cpp */
/* Texture::get_pixel (texture.cpp:56-62): BGR bytes -> Color3f{B,G,R}/255.  Byte offsets
 * outside the decoded buffer read as 0 (the reference reads out of bounds: undefined). */
static inline C3 tex_pixel(const pgrt_texture* t, int x, int y)
{
    C3 c = {0, 0, 0};
    int64_t off = (int64_t)y * t->pitch + (int64_t)x * t->bpp;
    int64_t size = (int64_t)t->pitch * t->height;
    if (off < 0 || off + 2 >= size) return c;
    c.r = t->data[off] / 255.0f;
    c.g = t->data[off + 1] / 255.0f;
    c.b = t->data[off + 2] / 255.0f;
    return c;
}

/* Texture::get_texel (texture.cpp:77-130), bilinear with the reference's edge quirks. */
static C3 tex_texel(const pgrt_texture* t, float u, float v)
{
    C3 black = {0, 0, 0};
    float x = u * (float)t->width;
    float y = v * (float)t->height;
    /* float->int of NaN or huge values is undefined in the reference: black */
    if (!(fabsf(x) < 16777216.0f) || !(fabsf(y) < 16777216.0f)) return black;
    int tmp_x1 = (int)floorf(x);
    int tmp_x2 = (int)ceilf(x);
    int tmp_y1 = (int)floorf(y);
    int tmp_y2 = (int)ceilf(y);
    int x1 = (tmp_x1 < 1) ? tmp_x1 + 1 : tmp_x1;
    int x2 = (tmp_x2 == t->width) ? 0 : tmp_x2;
    int y1 = (tmp_y1 < 1) ? tmp_y1 + 1 : tmp_y1;
    int y2 = (tmp_y2 == t->height) ? tmp_y1 : tmp_y2;
    if (x1 == x2 || y1 == y2) return black;
    C3 x1y1 = tex_pixel(t, x1, y1);
    C3 x2y1 = tex_pixel(t, x2, y1);
    C3 x1y2 = tex_pixel(t, x1, y2);
    C3 x2y2 = tex_pixel(t, x2, y2);
    float Q11 = ((float)x2 - x) / (float)(x2 - x1);
    float Q21 = (x - (float)x1) / (float)(x2 - x1);
    float Q12 = ((float)x2 - x) / (float)(x2 - x1);
    float Q22 = (x - (float)x1) / (float)(x2 - x1);
    C3 f1 = {x1y1.r * Q11 + x2y1.r * Q21, x1y1.g * Q11 + x2y1.g * Q21, x1y1.b * Q11 + x2y1.b * Q21};
    C3 f2 = {x1y2.r * Q12 + x2y2.r * Q22, x1y2.g * Q12 + x2y2.g * Q22, x1y2.b * Q12 + x2y2.b * Q22};
    float wy2 = ((float)y2 - y) / (float)(y2 - y1);
    float wy1 = (y - (float)y1) / (float)(y2 - y1);
    C3 out = {f1.r * wy2 + f2.r * wy1, f1.g * wy2 + f2.g * wy1, f1.b * wy2 + f2.b * wy1};
    return out;
}

/* SphericalMap::get_texel (SphericalMap.cpp:17-29) */
static C4 env_texel(const orc_scene* s, float x, float y, float z)
{
    C4 out = {0, 0, 0, 1};
    if (s->env < 0) return out;
    V3 vec = v_normalize(v3(x, z, y));
    float u = (float)(0.5 + (double)M_ATAN2F(vec.x, vec.z) / (2 * 3.14159265358979323846));
    float v = (float)(0.5 - (double)M_ASINF(vec.y) / 3.14159265358979323846);
    C3 c = tex_texel(&s->tex[s->env], u, v);
    out.r = c.b;
    out.g = c.g;
    out.b = c.r;
    out.a = 1;
    return out;
}

/* ------------------------------------------------------------------ utils.cpp:204-241 */
static float c_compress(float u)
{
    if (u <= 0) return 0.0f;
    if (u >= 1) return 1.0f;
    if ((double)u <= 0.00313080) return (float)(12.92 * (double)u);
    return (float)(1.00 * M_POWD((double)u, 1 / 2.4) - 0.055);
}
static float c_expand(float u)
{
    if (u <= 0) return 0.0f;
    if (u >= 1) return 1.0f;
    if ((double)u <= 0.04045) return (float)((double)u / 12.92);
    return (float)M_POWD(((double)u + 0.055) / 1.055, 2.4);
}
static C4 compress4(C4 c) { C4 o = {c_compress(c.b), c_compress(c.g), c_compress(c.r), 0.1f}; return o; }
static C4 expand4(C4 c) { C4 o = {c_expand(c.b), c_expand(c.g), c_expand(c.r), 0.1f}; return o; }
static C4 mix_linear(C4 c0, C4 c1, float a)
{
    C4 o = {a * c0.b + (1 - a) * c1.b, a * c0.g + (1 - a) * c1.g, a * c0.r + (1 - a) * c1.r, 1.0f};
    return o;
}
static C4 mix_srgb(C4 c0, C4 c1, float a) { return compress4(mix_linear(expand4(c0), expand4(c1), a)); }

/* Raytracer::gamma (raytracer.cpp:439-446): pow(c,g)*pow(c,g) with the r<->b swap */
static C4 gamma4(C4 in, float g)
{
    float b = M_POWF(in.b, g) * M_POWF(in.b, g);
    float gg = M_POWF(in.g, g) * M_POWF(in.g, g);
    float r = M_POWF(in.r, g) * M_POWF(in.r, g);
    C4 o = {b, gg, r, 1.0f};
    return o;
}

/* ------------------------------------------------------------------ raytracer.cpp */
typedef struct {
    uint64_t primary, shadow, reflect, refract, tests, visits; /* tests, visits adjacent */
} Counters;

/* Raytracer::is_illuminated + LightSource::GenerateRay (raytracer.cpp:150-176,
 * LightSource.cpp:11-32): the shadow ray starts AT the light and points along the hit
 * position vector H (unnormalized) with tfar = |L - H|; closest hit decides. */
static int is_illuminated(const orc_scene* s, const pgrt_light* L, V3 hit, V3 n, Counters* cn)
{
    V3 lp = v3(L->position[0], L->position[1], L->position[2]);
    if (v_dot(n, lp) < 0) return 0;
    Ray r;
    r.org = lp;
    r.dir = hit;
    r.tnear = 0.01f;
    r.tfar = v_len(v3(lp.x - hit.x, lp.y - hit.y, lp.z - hit.z));
    r.time = 0.0f;
    cn->shadow++;
    Hit h = scene_intersect(s, &r, &cn->tests);
    if (h.prim >= 0) {
        const pgrt_material* m = &s->mats[s->mat[h.prim]];
        return m->type == PGRT_MATERIAL_DIELECTRIC;
    }
    return 1;
}

/* get_reflection_ray (raytracer.cpp:209-235) */
static Ray reflection_ray(V3 d, V3 n, V3 hit, float ior)
{
    d = v_normalize(d);
    n = v_normalize(n);
    V3 rd = v_sub(d, v_scale(2, v_scale(v_dot(d, n), n)));
    Ray r;
    r.org = hit;
    r.dir = rd;
    r.tnear = 0.01f;
    r.tfar = FLT_MAX;
    r.time = ior;
    return r;
}

/* get_refraction_ray (raytracer.cpp:178-207); NaN direction on total internal reflection */
static Ray refraction_ray(V3 d, V3 n, float n1, float n2, V3 hit)
{
    d = v_normalize(d);
    n = v_normalize(n);
    float n1_n2 = n1 / n2;
    float d_n = v_dot(d, n);
    V3 sd = v3(d.x * n1_n2, d.y * n1_n2, d.z * n1_n2);
    float k = n1_n2 * d_n + sqrtf(1 - ((n1_n2 * n1_n2) * (1 - (d_n * d_n))));
    V3 rd = v_sub(sd, v_scale(k, n));
    Ray r;
    r.org = hit;
    r.dir = rd;
    r.tnear = 0.01f;
    r.tfar = FLT_MAX;
    r.time = n2;
    return r;
}

static C4 trace(const orc_scene* s, const Ray* ray, int level, int max_level, Counters* cn);

/* Phong branch (raytracer.cpp:325-385) */
static C4 shade_phong(const orc_scene* s, const Ray* ray, const pgrt_material* m, int prim,
                      float hu, float hv, V3 n, V3 hit, Counters* cn)
{
    float m_d_r, m_d_g, m_d_b;
    if (m->diffuse_tex < 0) {
        m_d_r = m->diffuse[2];
        m_d_g = m->diffuse[1];
        m_d_b = m->diffuse[0];
    } else {
        const float* t = s->uv + 6 * prim;
        float tu = interp1(t[0], t[2], t[4], hu, hv);
        float tv = interp1(t[1], t[3], t[5], hu, hv);
        C3 texel = tex_texel(&s->tex[m->diffuse_tex], tu, 1.0f - tv);
        m_d_r = texel.r;
        m_d_g = texel.g;
        m_d_b = texel.b;
    }
    float blue = 0, green = 0, red = 0;
    for (int li = 0; li < s->nlight; ++li) {
        const pgrt_light* L = &s->lights[li];
        if (!is_illuminated(s, L, hit, n, cn)) continue;
        V3 lv = v_normalize(v3(L->position[0] - hit.x, L->position[1] - hit.y, L->position[2] - hit.z));
        V3 cv = v_normalize(v3(ray->org.x - ray->dir.x, ray->org.y - ray->dir.y, ray->org.z - ray->dir.z));
        float gamma = m->shininess;
        float i_d_r = L->diffuse[2], i_d_g = L->diffuse[1], i_d_b = L->diffuse[0];
        float i_s_r = L->specular[2], i_s_g = L->specular[1], i_s_b = L->specular[0];
        float m_s_r = m->specular[2], m_s_g = m->specular[1], m_s_b = m->specular[0];
        float nl = v_dot(n, lv);
        V3 l_r = v_sub(v_scale(2 * nl, n), lv);
        l_r = v_normalize(l_r);
        float spec = M_POWF(v_dot(cv, l_r), gamma);
        blue += i_d_b * m_d_b * v_dot(n, lv) + i_s_b * m_s_b * spec;
        green += i_d_g * m_d_g * v_dot(n, lv) + i_s_g * m_s_g * spec;
        red += i_d_r * m_d_r * v_dot(n, lv) + i_s_r * m_s_r * spec;
    }
    C4 c = {blue, green, red, 1.0f};
    return c;
}

/* Raytracer::trace (raytracer.cpp:237-394) */
static C4 trace(const orc_scene* s, const Ray* ray, int level, int max_level, Counters* cn)
{
    Hit h = scene_intersect(s, ray, &cn->tests);
    V3 d = v_normalize(ray->dir);
    if (h.prim >= 0) {
        const float* nn = s->nrm + 9 * h.prim;
        V3 n = v3(interp1(nn[0], nn[3], nn[6], h.u, h.v), interp1(nn[1], nn[4], nn[7], h.u, h.v),
                  interp1(nn[2], nn[5], nn[8], h.u, h.v));
        const pgrt_material* m = &s->mats[s->mat[h.prim]];
        n = v_normalize(n);
        V3 hit = v_add(ray->org, v_scale(h.t, ray->dir));
        float n1, n2;
        if (ray->time == PGRT_IOR_AIR) { n1 = PGRT_IOR_AIR; n2 = m->ior; }
        else { n1 = m->ior; n2 = PGRT_IOR_AIR; }
        if (v_dot(n, d) > 0) n = v_neg(n);
        if (level >= max_level) { C4 k = {0, 0, 0, 1}; return k; }
        V3 v = v_neg(d);
        if (m->type == PGRT_MATERIAL_DIELECTRIC) {
            Ray rr = reflection_ray(d, n, hit, n1);
            cn->reflect++;
            C4 refl = trace(s, &rr, level + 1, max_level, cn);
            C4 att;
            att.r = M_EXPF(-(1 - m->diffuse[0]) * h.t);
            att.g = M_EXPF(-(1 - m->diffuse[1]) * h.t);
            att.b = M_EXPF(-(1 - m->diffuse[2]) * h.t);
            Ray tr = refraction_ray(d, n, n1, n2, hit);
            if (tr.dir.x == tr.dir.x) {
                cn->refract++;
                C4 refr = trace(s, &tr, level + 1, max_level, cn);
                float cos1 = fabsf(v_dot(n, v));
                float alpha = (n1 - n2) / (n1 + n2);
                float R = (float)((double)(alpha * alpha + (1 - (alpha * alpha))) *
                                  M_POWD((double)(1 - cos1), 5.0));
                C4 c = mix_srgb(refl, refr, R);
                C4 o = {c.r * att.r, c.g * att.g, c.b * att.b, 1};
                return o;
            }
            C4 o = {refl.r * att.r, refl.g * att.g, refl.b * att.b, 1};
            return o;
        }
        return shade_phong(s, ray, m, h.prim, h.u, h.v, n, hit, cn);
    }
    return env_texel(s, d.x, d.y, d.z);
}

static void jitter4(const pgrt_render_params* p, uint32_t pixel, uint32_t sample, float S,
                    float out[4])
{
    if (p->jitter == PGRT_JITTER_NONE) { out[0] = out[1] = out[2] = out[3] = 0.0f; return; }
    float ja = -0.5f / S, jb = 0.5f / S;
    float la = -p->aperture / 2.0f, lb = p->aperture / 2.0f;
    float u0 = pg_jitter_u01(p->seed, p->frame, pixel, sample, 0);
    float u1 = pg_jitter_u01(p->seed, p->frame, pixel, sample, 1);
    int corr = p->jitter == PGRT_JITTER_HASH_CORRELATED;
    float u2 = corr ? u0 : pg_jitter_u01(p->seed, p->frame, pixel, sample, 2);
    float u3 = corr ? u1 : pg_jitter_u01(p->seed, p->frame, pixel, sample, 3);
    out[0] = u0 * (jb - ja) + ja;
    out[1] = u1 * (jb - ja) + ja;
    out[2] = u2 * (lb - la) + la;
    out[3] = u3 * (lb - la) + la;
}

/* Raytracer::get_pixel (raytracer.cpp:396-437) */
static C4 get_pixel(const orc_scene* s, const Cam* k, const pgrt_render_params* p, int px, int py,
                    Counters* cn)
{
    const int S = p->spp_side;
    C4 sum = {0.0f, 0.0f, 0.0f, 1.0f};
    uint32_t pixel = (uint32_t)py * (uint32_t)k->width + (uint32_t)px;
    for (int sx = 0; sx < S; ++sx) {
        for (int sy = 0; sy < S; ++sy) {
            float j[4];
            jitter4(p, pixel, (uint32_t)(sx * S + sy), (float)S, j);
            float nx = (float)px + ((float)sx * (1.0f / (float)S)) + j[0];
            float ny = (float)py + ((float)sy * (1.0f / (float)S)) + j[1];
            Ray r = p->dof ? cam_ray_dof(k, nx, ny, p->focal_distance, j[2], j[3])
                           : cam_ray_pinhole(k, nx, ny);
            r.time = PGRT_IOR_AIR;
            cn->primary++;
            C4 c = trace(s, &r, 0, p->max_level, cn);
            sum.r += c.r;
            sum.g += c.g;
            sum.b += c.b;
        }
    }
    const int area = S * S;
    C4 in = {sum.b / (float)area, sum.g / (float)area, sum.r / (float)area, 1.0f};
    return gamma4(in, p->gamma_level);
}

/* ------------------------------------------------------------------ path tracing
 * PGRT_MODE_PATH: the "Whole pathtracing" item of the reference's README to-do list
 * (README.md:17-21).  The reference has no path tracer; the semantics are this project's
 * (DESIGN.md §2 "Path tracing") built from the reference's own pieces: trace()'s hit setup
 * (raytracer.cpp:241-288), the dielectric's reflection / refraction rays, attenuation and
 * Fresnel-like R (:294-316, :178-235), the Phong term of shade_phong (:355-382) and the
 * environment lookup on a miss (:390-393).  Per path, in this order per bounce b:
 *   miss                -> L += T * env(dir), end
 *   hit, b >= max_level -> end (raytracer.cpp:282-283)
 *   dielectric          -> T *= attenuation; reflect if TIR or u < R, else refract
 *   other               -> for every light with n . (Lp - H) > 0: a hard shadow ray from H
 *                          towards the light (tnear 0.01, tfar |Lp - H|; a dielectric occluder
 *                          lets the light through, raytracer.cpp:166-172); lit -> L += T * Phong
 *                          term; then T *= albedo and a cosine-weighted bounce (Malley's method,
 *                          rejection-sampled disk, Duff et al.'s orthonormal basis); T == 0 ends
 * Colours use trace()'s channel convention (C4.r carries Kd[0] / the texel's .b, as in
 * shade_phong's "blue" variable).  Random numbers: pg_path_u01 (pgrt_detmath.h). */

/* Building an orthonormal basis, revisited (Duff et al. 2017) */
static void onb(V3 n, V3* b1, V3* b2)
{
    const float sign = copysignf(1.0f, n.z);
    const float a = -1.0f / (sign + n.z);
    const float b = n.x * n.y * a;
    *b1 = v3(1.0f + sign * n.x * n.x * a, sign * b, -sign * n.x);
    *b2 = v3(b, sign + n.y * n.y * a, -n.y);
}

/* cosine-weighted direction about n: a uniform point of the unit disk (up to 8 rejection
 * candidates, else the pole) lifted to the hemisphere */
static V3 cosine_dir(uint32_t key, uint32_t bounce, V3 n)
{
    float x = 0.0f, y = 0.0f;
    for (uint32_t j = 0; j < 8u; ++j) {
        const float a = 2.0f * pg_path_u01(key, bounce, 1u + 2u * j) - 1.0f;
        const float c = 2.0f * pg_path_u01(key, bounce, 2u + 2u * j) - 1.0f;
        if (a * a + c * c < 1.0f) { x = a; y = c; break; }
    }
    const float z = sqrtf(1.0f - (x * x + y * y));
    V3 b1, b2;
    onb(n, &b1, &b2);
    return v3(x * b1.x + y * b2.x + z * n.x, x * b1.y + y * b2.y + z * n.y, x * b1.z + y * b2.z + z * n.z);
}

static C4 path_sample(const orc_scene* s, Ray r, int max_level, uint32_t key, Counters* cn)
{
    C4 L = {0.0f, 0.0f, 0.0f, 1.0f};
    float tr = 1.0f, tg = 1.0f, tb = 1.0f; /* throughput, C4 channel order */
    for (int b = 0;; ++b) {
        Hit h = scene_intersect(s, &r, &cn->tests);
        V3 d = v_normalize(r.dir);
        if (h.prim < 0) {
            C4 e = env_texel(s, d.x, d.y, d.z);
            L.r = L.r + tr * e.r;
            L.g = L.g + tg * e.g;
            L.b = L.b + tb * e.b;
            break;
        }
        const float* nn = s->nrm + 9 * h.prim;
        V3 n = v3(interp1(nn[0], nn[3], nn[6], h.u, h.v), interp1(nn[1], nn[4], nn[7], h.u, h.v),
                  interp1(nn[2], nn[5], nn[8], h.u, h.v));
        const pgrt_material* m = &s->mats[s->mat[h.prim]];
        n = v_normalize(n);
        V3 hit = v_add(r.org, v_scale(h.t, r.dir));
        float n1, n2;
        if (r.time == PGRT_IOR_AIR) { n1 = PGRT_IOR_AIR; n2 = m->ior; }
        else { n1 = m->ior; n2 = PGRT_IOR_AIR; }
        if (v_dot(n, d) > 0) n = v_neg(n);
        if (b >= max_level) break;
        if (m->type == PGRT_MATERIAL_DIELECTRIC) {
            Ray rr = reflection_ray(d, n, hit, n1);
            const float ar = M_EXPF(-(1 - m->diffuse[0]) * h.t);
            const float ag = M_EXPF(-(1 - m->diffuse[1]) * h.t);
            const float ab = M_EXPF(-(1 - m->diffuse[2]) * h.t);
            Ray fr = refraction_ray(d, n, n1, n2, hit);
            int refract = 0;
            if (fr.dir.x == fr.dir.x) { /* no total internal reflection */
                float cos1 = fabsf(v_dot(n, v_neg(d)));
                float alpha = (n1 - n2) / (n1 + n2);
                float R = (float)((double)(alpha * alpha + (1 - (alpha * alpha))) * M_POWD((double)(1 - cos1), 5.0));
                refract = !(pg_path_u01(key, (uint32_t)b, 0u) < R);
            }
            tr = tr * ar;
            tg = tg * ag;
            tb = tb * ab;
            if (refract) { r = fr; cn->refract++; }
            else { r = rr; cn->reflect++; }
            continue;
        }
        /* diffuse colour as shade_phong (raytracer.cpp:337-349) */
        float m_d_r, m_d_g, m_d_b;
        if (m->diffuse_tex < 0) {
            m_d_r = m->diffuse[2]; m_d_g = m->diffuse[1]; m_d_b = m->diffuse[0];
        } else {
            const float* t = s->uv + 6 * h.prim;
            float tu = interp1(t[0], t[2], t[4], h.u, h.v);
            float tv = interp1(t[1], t[3], t[5], h.u, h.v);
            C3 texel = tex_texel(&s->tex[m->diffuse_tex], tu, 1.0f - tv);
            m_d_r = texel.r; m_d_g = texel.g; m_d_b = texel.b;
        }
        for (int li = 0; li < s->nlight; ++li) { /* next-event estimation, hard shadows */
            const pgrt_light* Lt = &s->lights[li];
            V3 lp = v3(Lt->position[0], Lt->position[1], Lt->position[2]);
            V3 tol = v3(lp.x - hit.x, lp.y - hit.y, lp.z - hit.z);
            if (!(v_dot(n, tol) > 0)) continue;
            V3 lv = v_normalize(tol);
            Ray sr;
            sr.org = hit; sr.dir = lv; sr.tnear = 0.01f; sr.tfar = v_len(tol); sr.time = 0.0f;
            cn->shadow++;
            Hit sh = scene_intersect(s, &sr, &cn->tests);
            if (sh.prim >= 0 && s->mats[s->mat[sh.prim]].type != PGRT_MATERIAL_DIELECTRIC) continue;
            V3 cv = v_normalize(v3(r.org.x - r.dir.x, r.org.y - r.dir.y, r.org.z - r.dir.z));
            float i_d_r = Lt->diffuse[2], i_d_g = Lt->diffuse[1], i_d_b = Lt->diffuse[0];
            float i_s_r = Lt->specular[2], i_s_g = Lt->specular[1], i_s_b = Lt->specular[0];
            float m_s_r = m->specular[2], m_s_g = m->specular[1], m_s_b = m->specular[0];
            float nl = v_dot(n, lv);
            V3 l_r = v_sub(v_scale(2 * nl, n), lv);
            l_r = v_normalize(l_r);
            float spec = M_POWF(v_dot(cv, l_r), m->shininess);
            float blue = i_d_b * m_d_b * v_dot(n, lv) + i_s_b * m_s_b * spec;
            float green = i_d_g * m_d_g * v_dot(n, lv) + i_s_g * m_s_g * spec;
            float red = i_d_r * m_d_r * v_dot(n, lv) + i_s_r * m_s_r * spec;
            L.r = L.r + tr * blue;
            L.g = L.g + tg * green;
            L.b = L.b + tb * red;
        }
        tr = tr * m_d_b;
        tg = tg * m_d_g;
        tb = tb * m_d_r;
        if (!(tr > 0.0f || tg > 0.0f || tb > 0.0f)) break;
        V3 nd = cosine_dir(key, (uint32_t)b, n);
        Ray next;
        next.org = hit; next.dir = nd; next.tnear = 0.01f; next.tfar = FLT_MAX; next.time = r.time;
        r = next;
        cn->reflect++;
    }
    return L;
}

/* get_pixel (raytracer.cpp:396-437) with path_sample in place of trace */
static C4 get_pixel_path(const orc_scene* s, const Cam* k, const pgrt_render_params* p, int px, int py,
                         Counters* cn)
{
    const int S = p->spp_side;
    C4 sum = {0.0f, 0.0f, 0.0f, 1.0f};
    uint32_t pixel = (uint32_t)py * (uint32_t)k->width + (uint32_t)px;
    for (int sx = 0; sx < S; ++sx) {
        for (int sy = 0; sy < S; ++sy) {
            float j[4];
            const uint32_t sample = (uint32_t)(sx * S + sy);
            jitter4(p, pixel, sample, (float)S, j);
            float nx = (float)px + ((float)sx * (1.0f / (float)S)) + j[0];
            float ny = (float)py + ((float)sy * (1.0f / (float)S)) + j[1];
            Ray r = p->dof ? cam_ray_dof(k, nx, ny, p->focal_distance, j[2], j[3])
                           : cam_ray_pinhole(k, nx, ny);
            r.time = PGRT_IOR_AIR;
            cn->primary++;
            C4 c = path_sample(s, r, p->max_level, pg_path_key(p->seed, p->frame, pixel, sample), cn);
            sum.r += c.r;
            sum.g += c.g;
            sum.b += c.b;
        }
    }
    const int area = S * S;
    C4 in = {sum.b / (float)area, sum.g / (float)area, sum.r / (float)area, 1.0f};
    return gamma4(in, p->gamma_level);
}

/* ------------------------------------------------------------------ API */
orc_scene* orc_scene_create(const pgrt_scene_desc* d, int accel)
{
    if (!d || d->num_triangles < 0) return NULL;
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    int N = d->num_triangles;
    s->ntri = N;
    size_t n1 = (size_t)(N > 0 ? N : 1);
    s->pos = (float*)malloc(sizeof(float) * 9 * n1);
    s->nrm = (float*)malloc(sizeof(float) * 9 * n1);
    s->uv = (float*)malloc(sizeof(float) * 6 * n1);
    s->mat = (int*)malloc(sizeof(int) * n1);
    s->pre = (float*)malloc(sizeof(float) * 12 * n1);
    if (N > 0) {
        memcpy(s->pos, d->positions, sizeof(float) * 9 * (size_t)N);
        memcpy(s->nrm, d->normals, sizeof(float) * 9 * (size_t)N);
        memcpy(s->uv, d->uvs, sizeof(float) * 6 * (size_t)N);
        memcpy(s->mat, d->material_ids, sizeof(int) * (size_t)N);
    }
    s->nmat = d->num_materials;
    s->mats = (pgrt_material*)malloc(sizeof(pgrt_material) * (size_t)(s->nmat > 0 ? s->nmat : 1));
    if (s->nmat > 0) memcpy(s->mats, d->materials, sizeof(pgrt_material) * (size_t)s->nmat);
    s->ntex = d->num_textures;
    s->tex = (pgrt_texture*)malloc(sizeof(pgrt_texture) * (size_t)(s->ntex > 0 ? s->ntex : 1));
    s->texdata = (unsigned char**)calloc((size_t)(s->ntex > 0 ? s->ntex : 1), sizeof(unsigned char*));
    for (int i = 0; i < s->ntex; ++i) {
        s->tex[i] = d->textures[i];
        size_t bytes = (size_t)d->textures[i].pitch * (size_t)d->textures[i].height;
        s->texdata[i] = (unsigned char*)malloc(bytes ? bytes : 1);
        memcpy(s->texdata[i], d->textures[i].data, bytes);
        s->tex[i].data = s->texdata[i];
    }
    s->env = d->env_texture;
    s->nlight = d->num_lights;
    s->lights = (pgrt_light*)malloc(sizeof(pgrt_light) * (size_t)(s->nlight > 0 ? s->nlight : 1));
    if (s->nlight > 0) memcpy(s->lights, d->lights, sizeof(pgrt_light) * (size_t)s->nlight);
    /* a triangle whose material index is out of range shades with material 0 */
    for (int i = 0; i < N; ++i)
        if (s->mat[i] < 0 || s->mat[i] >= s->nmat) s->mat[i] = 0;
    tri_precompute(s);
    s->accel = accel;
    if (accel) bvh_build(s);
    return s;
}

void orc_scene_destroy(orc_scene* s)
{
    if (!s) return;
    free(s->pos); free(s->nrm); free(s->uv); free(s->mat); free(s->pre);
    free(s->mats);
    for (int i = 0; i < s->ntex; ++i) free(s->texdata[i]);
    free(s->texdata); free(s->tex); free(s->lights);
    free(s->nodes); free(s->perm);
    free(s);
}

int orc_render(const orc_scene* s, const pgrt_camera* cam, const pgrt_render_params* p,
               int row_step, int threads, float* rgba, pgrt_stats* st)
{
    if (!s || !cam || !p || !rgba || p->spp_side < 1 || row_step < 1) return PGRT_ERR_INVALID_ARGUMENT;
    if (s->nmat < 1 && s->ntri > 0) return PGRT_ERR_INVALID_ARGUMENT;
    Cam k = cam_make(cam);
    int rx = p->rect_x, ry = p->rect_y, rw = p->rect_w, rh = p->rect_h;
    if (rw <= 0 || rh <= 0) { rx = 0; ry = 0; rw = cam->width; rh = cam->height; }
    int nrows = (rh + row_step - 1) / row_step;
    uint64_t prim = 0, shd = 0, rfl = 0, rfr = 0, tst = 0, vis = 0;
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt) reduction(+ : prim, shd, rfl, rfr, tst, vis)
#endif
    for (int ri = 0; ri < nrows; ++ri) {
        Counters cn = {0, 0, 0, 0, 0, 0};
        int y = ry + ri * row_step;
        for (int x = rx; x < rx + rw; ++x) {
            C4 c = p->mode == PGRT_MODE_PATH ? get_pixel_path(s, &k, p, x, y, &cn) : get_pixel(s, &k, p, x, y, &cn);
            float* o = rgba + ((size_t)(y - ry) * (size_t)rw + (size_t)(x - rx)) * 4;
            o[0] = c.r; o[1] = c.g; o[2] = c.b; o[3] = c.a;
        }
        prim += cn.primary; shd += cn.shadow; rfl += cn.reflect; rfr += cn.refract; tst += cn.tests; vis += cn.visits;
    }
    (void)threads;
    if (st) {
        memset(st, 0, sizeof(*st));
        st->rays_primary = prim;
        st->rays_shadow = shd;
        st->rays_reflect = rfl;
        st->rays_refract = rfr;
        st->tri_tests = tst;
        st->node_visits = vis;
    }
    return PGRT_OK;
}

int orc_intersect(const orc_scene* s, const float* rays, int n, float* hits)
{
    if (!s || n < 0 || (n > 0 && (!rays || !hits))) return PGRT_ERR_INVALID_ARGUMENT;
    for (int i = 0; i < n; ++i) {
        const float* q = rays + 8 * (size_t)i;
        Ray r;
        r.org = v3(q[0], q[1], q[2]);
        r.tnear = q[3];
        r.dir = v3(q[4], q[5], q[6]);
        r.tfar = q[7];
        r.time = 0;
        Hit h = scene_intersect(s, &r, NULL);
        float* o = hits + 4 * (size_t)i;
        o[0] = h.t; o[1] = h.u; o[2] = h.v;
        memcpy(&o[3], &h.prim, 4);
    }
    return PGRT_OK;
}

void orc_camera_basis(const pgrt_camera* cam, float out[10])
{
    Cam k = cam_make(cam);
    out[0] = k.f_y;
    for (int i = 0; i < 9; ++i) out[1 + i] = k.m[i];
}

void orc_generate_ray(const pgrt_camera* cam, float x, float y, int dof, float focal,
                      float aperture, float lens_r1, float lens_r2, float out[9])
{
    (void)aperture;
    Cam k = cam_make(cam);
    Ray r = dof ? cam_ray_dof(&k, x, y, focal, lens_r1, lens_r2) : cam_ray_pinhole(&k, x, y);
    out[0] = r.org.x; out[1] = r.org.y; out[2] = r.org.z;
    out[3] = r.dir.x; out[4] = r.dir.y; out[5] = r.dir.z;
    out[6] = r.tnear; out[7] = r.tfar; out[8] = r.time;
}

void orc_get_texel(const pgrt_texture* t, float u, float v, float out[3])
{
    C3 c = tex_texel(t, u, v);
    out[0] = c.r; out[1] = c.g; out[2] = c.b;
}

void orc_env_texel(const pgrt_texture* t, float x, float y, float z, float out[4])
{
    orc_scene s;
    memset(&s, 0, sizeof(s));
    s.tex = (pgrt_texture*)t;
    s.ntex = 1;
    s.env = 0;
    C4 c = env_texel(&s, x, y, z);
    out[0] = c.r; out[1] = c.g; out[2] = c.b; out[3] = c.a;
}

void orc_mix_srgb(const float c0[4], const float c1[4], float alpha, float out[4])
{
    C4 a = {c0[0], c0[1], c0[2], c0[3]}, b = {c1[0], c1[1], c1[2], c1[3]};
    C4 c = mix_srgb(a, b, alpha);
    out[0] = c.r; out[1] = c.g; out[2] = c.b; out[3] = c.a;
}

void orc_gamma(const float c[4], float g, float out[4])
{
    C4 a = {c[0], c[1], c[2], c[3]};
    C4 o = gamma4(a, g);
    out[0] = o.r; out[1] = o.g; out[2] = o.b; out[3] = o.a;
}

float orc_compress(float u) { return c_compress(u); }
float orc_expand(float u) { return c_expand(u); }

void orc_jitter(uint32_t seed, uint32_t frame, uint32_t pixel, uint32_t sample, float out[4])
{
    for (uint32_t k = 0; k < 4; ++k) out[k] = pg_jitter_u01(seed, frame, pixel, sample, k);
}

/* host evaluation of include/pgrt_detmath.h, same layout as pgrt_selftest_math (tests only) */
void orc_detmath_eval(const float* in, int n, float* out)
{
    for (int i = 0; i < n; ++i) {
        const float a = in[2 * i], b = in[2 * i + 1];
        float* o = out + 8 * (size_t)i;
        o[0] = sqrtf(a);
        o[1] = a / b;
        o[2] = pg_powf(a, b);
        o[3] = pg_expf(a);
        o[4] = pg_atan2f(a, b);
        o[5] = pg_asinf(a);
        o[6] = 1 / sqrtf(a);
        o[7] = (float)pg_pow_d((double)a, (double)b);
    }
}

/* ------------------------------------------------------------------ reference RNG cost
 * The reference re-seeds a std::mt19937 from the wall clock for every sample, twice
 * (raytracer.cpp:407-410 before the pixel jitter, PinHoleCamera.cpp:77-80 before the lens
 * offset), and draws two uniform_real_distribution<float> values from each (one 32-bit output per
 * float draw, libstdc++ generate_canonical<float, 24>).  This restates that work -- MT19937
 * seeding (624-word init) and two tempered outputs (the first triggers the 624-word twist) -- n
 * times, for bench.py's CPU baseline to report the reseeding cost separately.
 * Returns a checksum of the outputs so the work is not optimised away. */
uint32_t orc_mt19937_reseed(int n, uint32_t seed)
{
    uint32_t mt[624];
    uint32_t acc = 0;
    for (int r = 0; r < n; ++r) {
        mt[0] = seed + (uint32_t)r;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        for (int i = 0; i < 624; ++i) { /* twist */
            uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        for (int k = 0; k < 2; ++k) {
            uint32_t y = mt[k];
            y ^= y >> 11;
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= y >> 18;
            acc ^= y;
        }
    }
    return acc;
}
