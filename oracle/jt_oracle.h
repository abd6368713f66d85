/*
 * jt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path (Princic-1837592/julia-raytracer, src/trace.jl,
 * src/bvh.jl, src/scene.jl, src/shading.jl, src/sampling.jl, src/geometry.jl, src/math.jl,
 * src/color.jl). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker / the timed CPU baseline — never as the product path.
 *
 * Parity status: the reference cannot run here (no Julia), ships no
 * tests or golden vectors, and draws from an unseeded thread-local Xoshiro RNG. The oracle is
 * pinned statistically against the reference's own render images/cornellbox_path.png
 * (tests/golden/) and structurally against BVH shapes derived from src/bvh.jl.
 */
#ifndef JT_ORACLE_H
#define JT_ORACLE_H

#include "../include/jtrace.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_counters {
    uint64_t paths, rays, light_queries, nodes, instances, prims, shades;
} or_counters;

/* make_scene_bvh (src/bvh.jl:66-88), independent of the product's host builder. */
int or_build_scene_bvh(const jt_scene* scene, int32_t high_quality, jt_scene_bvh* out);
void or_free_scene_bvh(jt_scene_bvh* bvh);

/* make_trace_lights (src/trace.jl:117-187). */
int or_make_lights(const jt_scene* scene, jt_lights* out);
void or_free_lights(jt_lights* lights);

/* trace_samples (src/trace.jl:215-274) over global samples [s0, s1) for all W*H pixels into
 * one running mean (one sample stream), weight 1/(s - first + 1). image: W*H*4, albedo/normal:
 * W*H*3, hits: W*H. Rows are split over nthreads pthreads. Returns 0 or a negative jt_status. */
int or_trace(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights,
             const jt_params* params, int32_t width, int32_t height, int32_t first,
             int32_t s0, int32_t s1, float* image, float* albedo, float* normal,
             int64_t* hits, int32_t nthreads, or_counters* counters);

/* Row-restricted variant: pixels of rows [row0, row1) only (bounded CPU samples), with 2^lk
 * sample streams (include/jtrace.h jt_trace_range): for lk > 0 the streams' running means live
 * in part_img (k*W*H*4), part_alb / part_nrm (k*W*H*3) and part_hits (k*W*H), stream-major, and
 * the rows' image / AOVs / hits are their combination after the range. */
int or_trace_rows(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights,
                  const jt_params* params, int32_t width, int32_t height, int32_t row0,
                  int32_t row1, int32_t first, int32_t s0, int32_t s1, float* image,
                  float* albedo, float* normal, int64_t* hits, int32_t lk, float* part_img,
                  float* part_alb, float* part_nrm, int64_t* part_hits, int32_t nthreads,
                  or_counters* counters);

/* The build's env_alias option (include/jtrace.h jt_set_option "env_alias"): environment lights
 * draw their texel through Vose alias tables instead of upper_bound (jt_oracle.c, "alias
 * tables"). Applies to contexts set up after the call (or_trace*). */
void or_set_env_alias(int32_t on);
/* that alias table of one CDF: keep[i] (probability of keeping column i), other[i] (0-based) */
int or_alias_table(const float* cdf, int32_t n, float* keep, int32_t* other);

/* Single-function known-answer entry points (tests/test_oracle_kat.py). */
int or_intersect_triangle(const float* o, const float* d, float tmin, float tmax,
                          const float* p1, const float* p2, const float* p3, float* out_uvt);
int or_intersect_bbox(const float* o, const float* d, float tmin, float tmax,
                      const float* bmin, const float* bmax);
float or_fresnel_dielectric(float eta, const float* normal, const float* outgoing);
void or_rng_first(uint64_t seed, int32_t pixel, int32_t sample, int32_t n, float* out);
void or_inverse_frame(const float* frame, int32_t non_rigid, float* out);
void or_srgb_to_rgb(const uint8_t* bytes, int32_t n, float* out);
/* wide-record property check (tests): records, non-conservative children, leaves, volume ratio x 1000 */
int or_wide_check(const jt_bvh_tree* tlas, const jt_bvh_tree* blas, int32_t nblas, int64_t* out);

#ifdef __cplusplus
}
#endif

#endif
