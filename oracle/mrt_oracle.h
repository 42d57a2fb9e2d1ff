/* oracle/mrt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference render path (Maraneshi/MiniRayTracer) in plain C, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the parity checker.  It is
 * never linked into, loaded by, or called from the product (miniraytracer_amd/libmrt.so).
 *
 * Pinning: tests/test_oracle_pinning.py checks it bit-for-bit against the reference's own code
 * (oracle/_ref/mrt_ref_exact, built from /root/reference by oracle/ref/build_ref.sh) through the
 * committed fixtures in tests/golden/ (PCG/sampler KATs, hit KATs, per-path radiance and ray
 * counts of stream-matched renders).
 */
#ifndef MRT_ORACLE_H
#define MRT_ORACLE_H
#include <stdint.h>
#include "../include/mrt_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_desc {
    uint32_t width, height, sqrt_samples, max_bounces;
    float max_luminance;
    uint32_t mode;   /* 0 draw(), 1 draw2() */
    uint64_t seed;   /* stream key seed */
    uint32_t threads;
    uint32_t y0, y1; /* row range to render (y1 = 0: all rows) */
} oracle_desc;

/* Render rows [y0,y1) of the image into rgb (W*H*4 floats, row 0 = bottom); optional per-path
 * radiance (W*H*ns*3, pixel-major [pixel][s]) and ray counts (W*H*ns).  Returns total rays. */
uint64_t oracle_render(const mrt_scene_view* v, const oracle_desc* d, float* rgb, float* path_rgb, uint32_t* path_rays);

/* The reference's own deterministic mode (-threads 1, main.cpp:347-382): ONE worker stream seeded
 * (initstate, initseq) = the worker seeds main() draws after select_scene (main.cpp:357-361, see
 * mrt_worker_seeds), tiles of tile_size in work_queue order; mode 0 = draw() over work_queue_seq
 * (tile -> row -> pixel -> sample), mode 1 = draw2() over work_queue_dynamic (sample-major passes
 * over the tiles).  rgb = W*H*4 floats (row 0 = bottom).  Returns G_rayCounter. */
uint64_t oracle_render_ref_order(const mrt_scene_view* v, const oracle_desc* d, uint32_t tile_size, uint64_t initstate, uint64_t initseq,
                                 float* rgb);

/* One path (pixel, sample): radiance -> out[3]; returns its ray count. */
uint32_t oracle_path(const mrt_scene_view* v, const oracle_desc* d, uint32_t x, uint32_t y, uint32_t s, float* out);

/* Closest hit of an arbitrary ray against v->root (PCG seeded (seed, 4242) for constant_volume):
 * returns 1/0 and t,p,n into rec[7]. */
int oracle_hit(const mrt_scene_view* v, const float* o, const float* dir, float time, int inside, uint64_t seed, float* rec);

/* PCG KAT helpers */
void oracle_pcg_stream(uint64_t initstate, uint64_t initseq, uint32_t n, uint32_t* out);
void oracle_samplers(uint64_t initstate, uint64_t initseq, uint32_t n, uint32_t which, float* out /* n*3 */);

#ifdef __cplusplus
}
#endif
#endif
