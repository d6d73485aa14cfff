/* oracle.h -- CPU restatement of the reference Whitted trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load liboracle.so.  The product (libpgrt.so) never links or calls it.
 *
 * Pinning: the reference itself is unbuildable here (every TU includes the Windows-only
 * stdafx.h -> tchar.h/d3d11.h/dinput.h, and the Embree and FreeImage runtimes are absent;
 * see DESIGN.md "Oracle").  The restatement is pinned by the reference's own known-answer
 * demos tutorial_1 (tutorials.cpp:29-139) and tutorial_2 (tutorials.cpp:170-178, data
 * test4.png), checked in tests/test_oracle.py; every other function is restated line by line
 * from the reference source cited at each definition in oracle.c.
 */
#ifndef PGRT_ORACLE_H_
#define PGRT_ORACLE_H_

#include "pgrt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* accel: 0 brute force (every triangle), 1 binned-SAH BVH (CPU) */
orc_scene* orc_scene_create(const pgrt_scene_desc* desc, int accel);
void orc_scene_destroy(orc_scene* s);

/* Render rows rect_y + k*row_step of the frame; other rows untouched.  threads<=0: all. */
int orc_render(const orc_scene* s, const pgrt_camera* cam, const pgrt_render_params* p,
               int row_step, int threads, float* rgba, pgrt_stats* st);
int orc_intersect(const orc_scene* s, const float* rays, int n, float* hits);

/* scalar probes for unit tests */
void orc_camera_basis(const pgrt_camera* cam, float out[10]); /* f_y, M row-major */
void orc_generate_ray(const pgrt_camera* cam, float x, float y, int dof, float focal,
                      float aperture, float lens_r1, float lens_r2, float out[9]);
void orc_get_texel(const pgrt_texture* t, float u, float v, float out[3]);
void orc_env_texel(const pgrt_texture* t, float x, float y, float z, float out[4]);
void orc_mix_srgb(const float c0[4], const float c1[4], float alpha, float out[4]);
void orc_gamma(const float c[4], float g, float out[4]);
float orc_compress(float u);
float orc_expand(float u);
void orc_jitter(uint32_t seed, uint32_t frame, uint32_t pixel, uint32_t sample, float out[4]);
int orc_uses_libm(void);
void orc_detmath_eval(const float* in_pairs, int n, float* out8);
/* n reseedings of std::mt19937 + two draws each (the reference's per-sample RNG work) */
uint32_t orc_mt19937_reseed(int n, uint32_t seed);

#ifdef __cplusplus
}
#endif
#endif
