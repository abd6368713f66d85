/*
 * jt_oracle.c — TEST INFRASTRUCTURE ONLY (see jt_oracle.h).
 *
 * A plain-C, line-by-line restatement of the reference hot path of
 * Princic-1837592/julia-raytracer (pure Julia 1.8.3). Every function cites the Julia
 * source it follows. It is written independently of the HIP product kernels
 * (julia-raytracer_amd/csrc) and is only ever used as the parity checker and as the timed
 * CPU baseline ("kind": "port").
 *
 * Float contract, shared with the product by specification only:
 *   - build with -ffp-contract=off: no FMA contraction; every expression is evaluated in the
 *     reference's source order (Julia never fuses without muladd/@fastmath);
 *   - Julia's NaN-propagating, signbit-aware min/max (base/math.jl) are restated exactly;
 *   - transcendentals (sin, cos, atan, acos, log, exp, pow) are evaluated in double and
 *     rounded once to float — Julia's own Float32 kernels evaluate in Float64, so this is the
 *     closest portable statement of its results;
 *   - the RNG is the build's counter-based PCG32 stream keyed by (seed, pixel, sample)
 *     because the reference's rand(Float32) is unseeded (src/sampling.jl:18).
 * Parity with the reference itself is statistical (tests/test_oracle_golden.py).
 */
#include "jt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- math (src/math.jl) */
typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;
typedef struct { v3 x, y, z, o; } fr3; /* Frame3f: columns x, y, z, o (src/math.jl:46) */
typedef struct { v3 c1, c2, c3; } m3;  /* Mat3f: three column Vec3f (src/math.jl:63) */

static const float pif = 3.14159265358979323846f; /* Float32(pi) (src/math.jl:13) */
static const float ray_eps = 0.0001f;             /* src/geometry.jl:34 */
static const float min_roughness = 0.03f * 0.03f; /* src/scene.jl:46 */

static inline v2 V2(float x, float y) { v2 r = {x, y}; return r; }
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scl3(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 div3s(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline int eq3(v3 a, v3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
static inline int iszero3(v3 a) { return a.x == 0 && a.y == 0 && a.z == 0; }
static inline int isfinite3(v3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }
static inline v4 add4(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline v4 scl4(v4 a, float s) { return V4(a.x * s, a.y * s, a.z * s, a.w * s); }
static inline v3 xyz(v4 a) { return V3(a.x, a.y, a.z); }

/* dot(a, b) = sum(a .* b): left fold (src/math.jl:69) */
static inline float dot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* cross (src/math.jl:112) */
static inline v3 cross3(v3 a, v3 b) {
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* normalize (src/math.jl:71-78): divide by the length, zero stays zero */
static inline v3 normalize3(v3 a) {
    float l = sqrtf(dot3(a, a));
    return l != 0 ? div3s(a, l) : a;
}
static inline float length3(v3 a) { return sqrtf(dot3(a, a)); }
static inline float distance_squared(v3 a, v3 b) { v3 d = sub3(a, b); return dot3(d, d); }

/* Julia min/max for floats: NaN-propagating and signbit-aware (base/math.jl, Julia 1.8). */
static inline float jl_min(float x, float y) {
    int c = (y < x) || (signbit(y) && !signbit(x));
    return c ? (isnan(x) ? x : y) : (isnan(y) ? y : x);
}
static inline float jl_max(float x, float y) {
    int c = (y > x) || (!signbit(y) && signbit(x));
    return c ? (isnan(x) ? x : y) : (isnan(y) ? y : x);
}
/* clamp(x, lo, hi) = ifelse(x > hi, hi, ifelse(x < lo, lo, x)) (base/math.jl) */
static inline float jl_clamp(float x, float lo, float hi) { return x > hi ? hi : (x < lo ? lo : x); }
static inline long jl_clampi(long x, long lo, long hi) { return x > hi ? hi : (x < lo ? lo : x); }
static inline float max3f(v3 a) { return jl_max(jl_max(a.x, a.y), a.z); } /* maximum(v) */

/* transcendentals: evaluated in double, rounded once (float contract above) */
static inline float jl_sin(float x) { return (float)sin((double)x); }
static inline float jl_cos(float x) { return (float)cos((double)x); }
static inline float jl_atan(float x) { return (float)atan((double)x); }
static inline float jl_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
static inline float jl_acos(float x) { return (float)acos((double)x); }
static inline float jl_log(float x) { return (float)log((double)x); }
static inline float jl_exp(float x) { return (float)exp((double)x); }
static inline float jl_pow(float x, float y) { return (float)pow((double)x, (double)y); }

/* transform_point / transform_vector / transform_direction (src/math.jl:80-87) */
static inline v3 transform_point(const fr3* f, v3 p) {
    return add3(add3(add3(scl3(f->x, p.x), scl3(f->y, p.y)), scl3(f->z, p.z)), f->o);
}
static inline v3 transform_vector(const fr3* f, v3 b) {
    return add3(add3(scl3(f->x, b.x), scl3(f->y, b.y)), scl3(f->z, b.z));
}
static inline v3 transform_direction(const fr3* f, v3 b) { return normalize3(transform_vector(f, b)); }
/* Base.:*(m::Mat3f, f::Vec3f) (src/math.jl:105) */
static inline v3 m3_mul(const m3* m, v3 f) {
    return add3(add3(scl3(m->c1, f.x), scl3(m->c2, f.y)), scl3(m->c3, f.z));
}
static inline v3 m3_transform_direction(const m3* m, v3 b) { return normalize3(m3_mul(m, b)); }
/* transform_normal(frame, b, non_rigid=false) = normalize(transform_vector) (src/math.jl:124) */
static inline v3 transform_normal(const fr3* f, v3 b) { return normalize3(transform_vector(f, b)); }

static inline m3 transpose3(const m3* m) {
    m3 r;
    r.c1 = V3(m->c1.x, m->c2.x, m->c3.x);
    r.c2 = V3(m->c1.y, m->c2.y, m->c3.y);
    r.c3 = V3(m->c1.z, m->c2.z, m->c3.z);
    return r;
}
/* inverse(frame, non_rigid) (src/math.jl:95-103), inverse(Mat3f) = adjoint * (1/det) :107 */
static fr3 inverse_frame(const fr3* f, int non_rigid) {
    m3 rot = {f->x, f->y, f->z};
    m3 minv;
    if (non_rigid) {
        m3 cof = {cross3(rot.c2, rot.c3), cross3(rot.c3, rot.c1), cross3(rot.c1, rot.c2)};
        m3 adj = transpose3(&cof);
        float det = dot3(rot.c1, cross3(rot.c2, rot.c3));
        float s = 1.0f / det;
        minv.c1 = scl3(adj.c1, s);
        minv.c2 = scl3(adj.c2, s);
        minv.c3 = scl3(adj.c3, s);
    } else {
        minv = transpose3(&rot);
    }
    fr3 r;
    r.x = minv.c1;
    r.y = minv.c2;
    r.z = minv.c3;
    r.o = neg3(m3_mul(&minv, f->o));
    return r;
}
/* reflect / refract (src/math.jl:131-142) */
static inline v3 reflect3(v3 w, v3 n) { return add3(neg3(w), scl3(n, 2 * dot3(n, w))); }
static inline v3 refract3(v3 w, v3 n, float inv_eta) {
    float cosine = dot3(n, w);
    float k = 1 + inv_eta * inv_eta * (cosine * cosine - 1);
    if (k < 0) return V3(0, 0, 0);
    return add3(scl3(neg3(w), inv_eta), scl3(n, inv_eta * cosine - sqrtf(k)));
}
static inline fr3 frame_from(const float* a) {
    fr3 f;
    f.x = V3(a[0], a[1], a[2]);
    f.y = V3(a[3], a[4], a[5]);
    f.z = V3(a[6], a[7], a[8]);
    f.o = V3(a[9], a[10], a[11]);
    return f;
}

/* ----------------------------------------------------------- color (src/color.jl) */
static inline float srgb_to_rgb1(float c) {
    return c <= 0.04045f ? c / 12.92f : jl_pow((c + 0.055f) / 1.055f, 2.4f);
}

/* ------------------------------------------------------------------------ RNG (build) */
typedef struct { uint64_t state, inc; } rng_t;
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static inline rng_t rng_init(uint64_t seed, int32_t pixel, int32_t sample) {
    uint64_t key = mix64(seed ^ mix64(((uint64_t)(uint32_t)pixel << 32) | (uint64_t)(uint32_t)sample));
    rng_t r;
    r.inc = (mix64(key ^ 0xda3e39cb94b95bdbULL) << 1) | 1ULL;
    r.state = (r.inc + key) * 6364136223846793005ULL + r.inc;
    return r;
}
static inline uint32_t rng_next(rng_t* r) {
    uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18) ^ old) >> 27);
    uint32_t rot = (uint32_t)(old >> 59);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}
/* rand(Float32) in [0,1) with 24-bit resolution, like Julia's (src/sampling.jl:18) */
static inline float rand1f(rng_t* r) { return (float)(rng_next(r) >> 8) * 0x1.0p-24f; }
static inline v2 rand2f(rng_t* r) { float a = rand1f(r); float b = rand1f(r); return V2(a, b); }

/* --------------------------------------------------------------- sampling.jl */
static inline v2 sample_disk(v2 ruv) { /* src/sampling.jl:12-16 */
    float r = sqrtf(ruv.y);
    float phi = 2 * pif * ruv.x;
    return V2(jl_cos(phi) * r, jl_sin(phi) * r);
}
static inline float sample_hemisphere_cos_pdf(v3 normal, v3 direction) { /* :24-27 */
    float cosw = dot3(normal, direction);
    return cosw <= 0 ? 0 : cosw / pif;
}
static inline long sample_uniform(long size, float r) { /* :29, returns 1-based */
    return jl_clampi((long)truncf(r * (float)size) + 1, 1, size);
}
static inline float sample_uniform_pdf(long size) { return (float)(1.0 / (double)size); } /* :31 */
static long upper_bound(const float* cdf, long n, float limit) { /* :42-56, 1-based */
    long idx = 0, l = 1, r = n;
    while (l <= r) {
        long m = (l + r) / 2;
        if (cdf[m - 1] > limit) { idx = m; r = m - 1; }
        else l = m + 1;
    }
    return idx;
}
static inline long sample_discrete(const float* cdf, long n, float r) { /* :33-37, 1-based */
    float last = cdf[n - 1];
    r = jl_clamp(r * last, 0.0f, last - 0.00001f);
    long idx = upper_bound(cdf, n, r);
    return jl_clampi(idx, 1, n);
}
static inline float sample_discrete_pdf(const float* cdf, long idx1) { /* :39-40 */
    return idx1 == 1 ? cdf[0] : cdf[idx1 - 1] - cdf[idx1 - 2];
}
static inline v2 sample_triangle(v2 ruv) { /* :58 */
    return V2(1 - sqrtf(ruv.x), ruv.y * sqrtf(ruv.x));
}

/* --------------------------------------------------------------- geometry.jl */
typedef struct { v3 o, d; float tmin, tmax; } ray3;
typedef struct { v2 uv; float distance; int hit; } prim_isec;

static inline ray3 make_ray(v3 o, v3 d) { ray3 r = {o, d, ray_eps, INFINITY}; return r; }

/* intersect_bbox (src/geometry.jl:96-105): t1 *= 1.00000024 is a Float64 literal */
static inline int intersect_bbox(const ray3* ray, v3 dinv, const float* bmin, const float* bmax) {
    float mx = (bmin[0] - ray->o.x) * dinv.x, my = (bmin[1] - ray->o.y) * dinv.y,
          mz = (bmin[2] - ray->o.z) * dinv.z;
    float Mx = (bmax[0] - ray->o.x) * dinv.x, My = (bmax[1] - ray->o.y) * dinv.y,
          Mz = (bmax[2] - ray->o.z) * dinv.z;
    float tminx = jl_min(mx, Mx), tminy = jl_min(my, My), tminz = jl_min(mz, Mz);
    float tmaxx = jl_max(mx, Mx), tmaxy = jl_max(my, My), tmaxz = jl_max(mz, Mz);
    float t0 = jl_max(jl_max(jl_max(tminx, tminy), tminz), ray->tmin);
    float t1 = jl_min(jl_min(jl_min(tmaxx, tmaxy), tmaxz), ray->tmax);
    double t1d = (double)t1 * 1.00000024;
    return (double)t0 <= t1d;
}
/* intersect_triangle (src/geometry.jl:206-236) */
static inline prim_isec intersect_triangle(const ray3* ray, v3 p1, v3 p2, v3 p3) {
    prim_isec miss = {{0, 0}, INFINITY, 0};
    v3 edge1 = sub3(p2, p1), edge2 = sub3(p3, p1);
    v3 pvec = cross3(ray->d, edge2);
    float det = dot3(edge1, pvec);
    if (det == 0) return miss;
    float inv_det = 1.0f / det;
    v3 tvec = sub3(ray->o, p1);
    float u = dot3(tvec, pvec) * inv_det;
    if (u < 0 || u > 1) return miss;
    v3 qvec = cross3(tvec, edge1);
    float v = dot3(ray->d, qvec) * inv_det;
    if (v < 0 || u + v > 1) return miss;
    float t = dot3(edge2, qvec) * inv_det;
    if (t < ray->tmin || t > ray->tmax) return miss;
    prim_isec h = {{u, v}, t, 1};
    return h;
}
/* intersect_quad (src/geometry.jl:238-258) */
static inline prim_isec intersect_quad(const ray3* ray, v3 p1, v3 p2, v3 p3, v3 p4) {
    if (eq3(p3, p4)) return intersect_triangle(ray, p1, p2, p4);
    prim_isec i1 = intersect_triangle(ray, p1, p2, p4);
    prim_isec i2 = intersect_triangle(ray, p3, p4, p2);
    if (i2.hit) i2.uv = V2(1 - i2.uv.x, 1 - i2.uv.y);
    return i1.distance < i2.distance ? i1 : i2;
}
static inline v3 triangle_normal(v3 p1, v3 p2, v3 p3) { /* :262 */
    return normalize3(cross3(sub3(p2, p1), sub3(p3, p1)));
}
static inline float triangle_area(v3 p0, v3 p1, v3 p2) { /* :264 */
    return length3(cross3(sub3(p1, p0), sub3(p2, p0))) / 2;
}
static inline v3 quad_normal(v3 p1, v3 p2, v3 p3, v3 p4) { /* :267 */
    return normalize3(add3(triangle_normal(p1, p2, p4), triangle_normal(p3, p4, p2)));
}
static inline float quad_area(v3 p0, v3 p1, v3 p2, v3 p3) { /* :270 */
    return triangle_area(p0, p1, p3) + triangle_area(p2, p3, p1);
}
/* interpolate_triangle: @. p1 * (1 - u - v) + p2 * u + p3 * v (:275) */
static inline v3 interp_tri3(v3 p1, v3 p2, v3 p3, v2 uv) {
    float w = (1 - uv.x) - uv.y;
    return add3(add3(scl3(p1, w), scl3(p2, uv.x)), scl3(p3, uv.y));
}
static inline v2 interp_tri2(v2 p1, v2 p2, v2 p3, v2 uv) {
    float w = (1 - uv.x) - uv.y;
    return V2((p1.x * w + p2.x * uv.x) + p3.x * uv.y, (p1.y * w + p2.y * uv.x) + p3.y * uv.y);
}
static inline v4 interp_tri4(v4 p1, v4 p2, v4 p3, v2 uv) {
    float w = (1 - uv.x) - uv.y;
    return add4(add4(scl4(p1, w), scl4(p2, uv.x)), scl4(p3, uv.y));
}
/* interpolate_quad (:278-283) */
static inline v3 interp_quad3(v3 p1, v3 p2, v3 p3, v3 p4, v2 uv) {
    if (uv.x + uv.y <= 1) return interp_tri3(p1, p2, p4, uv);
    return interp_tri3(p3, p4, p2, V2(1 - uv.x, 1 - uv.y));
}
static inline v2 interp_quad2(v2 p1, v2 p2, v2 p3, v2 p4, v2 uv) {
    if (uv.x + uv.y <= 1) return interp_tri2(p1, p2, p4, uv);
    return interp_tri2(p3, p4, p2, V2(1 - uv.x, 1 - uv.y));
}
static inline v4 interp_quad4(v4 p1, v4 p2, v4 p3, v4 p4, v2 uv) {
    if (uv.x + uv.y <= 1) return interp_tri4(p1, p2, p4, uv);
    return interp_tri4(p3, p4, p2, V2(1 - uv.x, 1 - uv.y));
}
/* triangle_tangents_fromuv / quad_tangents_fromuv (:285-332) */
static void triangle_tangents_fromuv(v3 p1, v3 p2, v3 p3, v2 uv1, v2 uv2, v2 uv3, v3* tu, v3* tv) {
    v3 p = sub3(p2, p1), q = sub3(p3, p1);
    v2 s = V2(uv2.x - uv1.x, uv3.x - uv1.x);
    v2 t = V2(uv2.y - uv1.y, uv3.y - uv1.y);
    float div = s.x * t.y - s.y * t.x;
    if (div != 0) {
        *tu = div3s(V3(t.y * p.x - t.x * q.x, t.y * p.y - t.x * q.y, t.y * p.z - t.x * q.z), div);
        *tv = div3s(V3(s.x * q.x - s.y * p.x, s.x * q.y - s.y * p.y, s.x * q.z - s.y * p.z), div);
    } else {
        *tu = V3(1, 0, 0);
        *tv = V3(0, 1, 0);
    }
}

/* wide records of one binary tree (JT_TRAVERSAL_WIDE, see intersect_scene_wide) */
typedef struct {
    float o[3], s[3];
    int a[3];                          /* N's split axis, then L's and R's (0 for a leaf) */
    unsigned char lo[3][4], hi[3][4];  /* per axis, per slot */
    int child[4];                      /* binary node of the slot, -1 empty */
    int rec[4];                        /* record of an internal child, -1 otherwise */
} wrec_t;
typedef struct { int n, cap; wrec_t* r; } wtree_t;

/* ---------------------------------------------------------- scene view */
typedef struct ctx_s {
    const jt_scene* scene;
    const jt_scene_bvh* bvh;
    const jt_lights* lights;
    const jt_params* params;
    fr3* inst_frame;   /* InstanceData.frame */
    fr3* inst_inverse; /* inverse(frame, true), recomputed per visit by the reference */
    fr3* env_frame;
    fr3* env_inverse;  /* inverse(frame) rigid (src/scene.jl:906) */
    wtree_t wtlas;     /* JT_TRAVERSAL_WIDE: the TLAS's wide records */
    wtree_t* wblas;    /* and every BLAS's */
    fr3 camera_frame;
    float camera_aspect; /* cam.aspect, or W/H when --width/--height are given (see setup_ctx) */
    /* the build's env_alias option (or_set_env_alias): per light, its alias table or NULL */
    float** alias_keep;
    int32_t** alias_other;
    int width, height;
} ctx_t;

typedef struct {
    int32_t* stack;
    int32_t* sub_stack;
    int stack_size;
    int overflow;
    or_counters cnt;
    /* or_order_diff (diagnostic): the same scene query in another traversal order, compared */
    const struct ctx_s* alt;
    uint64_t diag[10];
    int path_diff;
    int tie;  /* the current near-first query accepted a hit at exactly its tmax */
} scratch_t;

static inline v3 pos3(const jt_shape* s, int32_t v) {
    return V3(s->positions[3 * v], s->positions[3 * v + 1], s->positions[3 * v + 2]);
}
static inline v3 nrm3(const jt_shape* s, int32_t v) {
    return V3(s->normals[3 * v], s->normals[3 * v + 1], s->normals[3 * v + 2]);
}
static inline v2 tc2(const jt_shape* s, int32_t v) { return V2(s->texcoords[2 * v], s->texcoords[2 * v + 1]); }
static inline v4 col4(const jt_shape* s, int32_t v) {
    return V4(s->colors[4 * v], s->colors[4 * v + 1], s->colors[4 * v + 2], s->colors[4 * v + 3]);
}

/* ------------------------------------------------------- BVH traversal (src/bvh.jl) */
typedef struct { int element; v2 uv; float distance; int hit; } shape_isec;
typedef struct { int instance, element; v2 uv; float distance; int hit; } scene_isec;

/* Exact-t ties in the near-first orders (the build's JT_TRAVERSAL_NEAR / WIDE, include/jtrace.h).
 * The reference accepts a hit at t == tmax (src/geometry.jl:226), so among equal-t hits the one
 * it tests last wins, which depends on its child order. A near-first query that accepts a hit at
 * exactly its current tmax (sc->tie) is run again in the reference's child order (flip 0: the same
 * records visited far child first) and reports that query's hit: the reference's own resolution.
 * `flip` below: 1 visits the near child first (the build's extension), 0 the reference's order. */
static inline void note_tie(scratch_t* sc, float t, float tmax) { if (t == tmax) sc->tie = 1; }

/* intersect_shape_bvh (src/bvh.jl:373-491), find_any = false */
static shape_isec intersect_shape_bvh(const ctx_t* c, int shape_id, ray3 ray, scratch_t* sc, int flip) {
    shape_isec isec = {-1, {0, 0}, 0, 0};
    const jt_bvh_tree* bvh = &c->bvh->blas[shape_id];
    const jt_shape* shape = &c->scene->shapes[shape_id];
    if (bvh->nnodes == 0) return isec;
    int32_t* stack = sc->sub_stack;
    int node_cur = 0; /* number of entries (Julia node_cur - 1) */
    stack[node_cur++] = 0;
    v3 dinv = V3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    /* ray_dsign; JT_TRAVERSAL_NEAR (build extension, include/jtrace.h) inverts the push order */
    int dsign[3] = {(ray.d.x < 0) ^ flip, (ray.d.y < 0) ^ flip, (ray.d.z < 0) ^ flip};
    while (node_cur != 0) {
        const jt_bvh_node* node = &bvh->nodes[stack[--node_cur]];
        sc->cnt.nodes++;
        if (!intersect_bbox(&ray, dinv, node->bmin, node->bmax)) continue;
        if (node->internal) {
            if (node_cur + 2 > sc->stack_size) { sc->overflow = 1; return isec; }
            if (dsign[node->axis] == 0) {
                stack[node_cur++] = node->start;
                stack[node_cur++] = node->start + 1;
            } else {
                stack[node_cur++] = node->start + 1;
                stack[node_cur++] = node->start;
            }
        } else if (shape->ntriangles > 0) {
            for (int i = node->start; i < node->start + node->num; i++) {
                int e = bvh->primitives[i];
                const int32_t* t = &shape->triangles[3 * e];
                sc->cnt.prims++;
                prim_isec p = intersect_triangle(&ray, pos3(shape, t[0]), pos3(shape, t[1]), pos3(shape, t[2]));
                if (!p.hit) continue;
                note_tie(sc, p.distance, ray.tmax);
                isec.element = e;
                isec.uv = p.uv;
                isec.distance = p.distance;
                isec.hit = 1;
                ray.tmax = p.distance;
            }
        } else if (shape->nquads > 0) {
            for (int i = node->start; i < node->start + node->num; i++) {
                int e = bvh->primitives[i];
                const int32_t* q = &shape->quads[4 * e];
                sc->cnt.prims++;
                prim_isec p = intersect_quad(&ray, pos3(shape, q[0]), pos3(shape, q[1]), pos3(shape, q[2]),
                                             pos3(shape, q[3]));
                if (!p.hit) continue;
                note_tie(sc, p.distance, ray.tmax);
                isec.element = e;
                isec.uv = p.uv;
                isec.distance = p.distance;
                isec.hit = 1;
                ray.tmax = p.distance;
            }
        }
    }
    return isec;
}

/* transform_ray (src/geometry.jl:107-111) */
static inline ray3 transform_ray(const fr3* f, const ray3* r) {
    ray3 o = {transform_point(f, r->o), transform_vector(f, r->d), r->tmin, r->tmax};
    return o;
}

/* intersect_scene_bvh (src/bvh.jl:306-371), find_any = false */
static scene_isec intersect_scene_bvh(const ctx_t* c, ray3 ray, scratch_t* sc, int flip) {
    scene_isec isec = {-1, -1, {0, 0}, 0, 0};
    const jt_bvh_tree* bvh = &c->bvh->tlas;
    if (bvh->nnodes == 0) return isec;
    int32_t* stack = sc->stack;
    int node_cur = 0;
    stack[node_cur++] = 0;
    v3 dinv = V3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    /* ray_dsign; JT_TRAVERSAL_NEAR (build extension, include/jtrace.h) inverts the push order */
    int dsign[3] = {(ray.d.x < 0) ^ flip, (ray.d.y < 0) ^ flip, (ray.d.z < 0) ^ flip};
    while (node_cur != 0) {
        const jt_bvh_node* node = &bvh->nodes[stack[--node_cur]];
        sc->cnt.nodes++;
        if (!intersect_bbox(&ray, dinv, node->bmin, node->bmax)) continue;
        if (node->internal) {
            if (node_cur + 2 > sc->stack_size) { sc->overflow = 1; return isec; }
            if (dsign[node->axis] == 0) {
                stack[node_cur++] = node->start;
                stack[node_cur++] = node->start + 1;
            } else {
                stack[node_cur++] = node->start + 1;
                stack[node_cur++] = node->start;
            }
        } else {
            for (int i = node->start; i < node->start + node->num; i++) {
                int inst_id = bvh->primitives[i];
                const jt_instance* inst = &c->scene->instances[inst_id];
                sc->cnt.instances++;
                ray3 inv_ray = transform_ray(&c->inst_inverse[inst_id], &ray);
                shape_isec s = intersect_shape_bvh(c, inst->shape, inv_ray, sc, flip);
                if (!s.hit) continue;
                isec.instance = inst_id;
                isec.element = s.element;
                isec.uv = s.uv;
                isec.distance = s.distance;
                isec.hit = 1;
                ray.tmax = s.distance;
            }
        }
    }
    return isec;
}

/* intersect_instance_bvh (src/bvh.jl:493-520) */
static scene_isec intersect_instance_bvh(const ctx_t* c, int inst_id, ray3 ray, scratch_t* sc, int flip) {
    scene_isec isec = {-1, -1, {0, 0}, 0, 0};
    const jt_instance* inst = &c->scene->instances[inst_id];
    sc->cnt.instances++;
    ray3 inv_ray = transform_ray(&c->inst_inverse[inst_id], &ray);
    shape_isec s = intersect_shape_bvh(c, inst->shape, inv_ray, sc, flip);
    if (!s.hit) return isec;
    isec.instance = inst_id;
    isec.element = s.element;
    isec.uv = s.uv;
    isec.distance = s.distance;
    isec.hit = 1;
    return isec;
}

/* ------------------------------------------------- wide traversal (JT_TRAVERSAL_WIDE) */
/* The build's 4-wide traversal (include/jtrace.h JT_TRAVERSAL_WIDE), restated from
 * its specification independently of the product's builder (jt_trace.hip build_wide): a record
 * per internal binary node N (or the root leaf) holding N's grandchildren in slots [LL, LR, RL,
 * RR] (a leaf child alone in its pair's first slot), their boxes quantised to bytes relative to
 * N's box, visited near child first in the binary DFS order; every record's children are tested
 * when the record is visited. Its closest hits equal the binary traversal's up to exact-t ties
 * and boxes the exact slab test culls by rounding (the quantised boxes are conservative). */

static float w_scale(int e) { /* 2^(e - 127), e a normal float's biased exponent */
    uint32_t b = (uint32_t)e << 23;
    float f;
    memcpy(&f, &b, 4);
    return f;
}
/* the largest lo with o + lo*s <= cmin and the smallest hi with o + hi*s >= cmax, in float */
static int w_quantize(float o, float s, float cmin, float cmax, unsigned* lo, unsigned* hi) {
    double f = floor(((double)cmin - (double)o) / (double)s);
    int q = (int)(f < 0 ? 0 : f > 255 ? 255 : f);
    while (q > 0 && o + (float)q * s > cmin) q--;
    while (q < 255 && o + (float)(q + 1) * s <= cmin) q++;
    if (!(o + (float)q * s <= cmin)) return 0;
    *lo = (unsigned)q;
    f = ceil(((double)cmax - (double)o) / (double)s);
    q = (int)(f < 0 ? 0 : f > 255 ? 255 : f);
    while (q < 255 && o + (float)q * s < cmax) q++;
    while (q > 0 && o + (float)(q - 1) * s >= cmax) q--;
    if (!(o + (float)q * s >= cmax)) return 0;
    *hi = (unsigned)q;
    return 1;
}
static int w_add(wtree_t* t) {
    if (t->n == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 64;
        t->r = (wrec_t*)realloc(t->r, sizeof(wrec_t) * (size_t)t->cap);
        if (!t->r) return -1;
    }
    return t->n++;
}
/* record of binary node `node` (and, recursively, of its internal grandchildren) */
static int w_build(const jt_bvh_tree* b, int node, wtree_t* t) {
    int r = w_add(t);
    if (r < 0) return -1;
    const jt_bvh_node* N = &b->nodes[node];
    if (!N->internal && N->num <= 0) { /* an empty tree (no boxes): a record without children */
        memset(&t->r[r], 0, sizeof(wrec_t));
        for (int k = 0; k < 4; k++) t->r[r].child[k] = t->r[r].rec[k] = -1;
        return r;
    }
    int slot[4] = {-1, -1, -1, -1}, a1 = 0, a2 = 0;
    if (!N->internal) {
        slot[0] = node;
    } else {
        const jt_bvh_node* L = &b->nodes[N->start];
        const jt_bvh_node* R = &b->nodes[N->start + 1];
        if (L->internal) { slot[0] = L->start; slot[1] = L->start + 1; a1 = L->axis; } else slot[0] = N->start;
        if (R->internal) { slot[2] = R->start; slot[3] = R->start + 1; a2 = R->axis; } else slot[2] = N->start + 1;
    }
    wrec_t w;
    memset(&w, 0, sizeof w);
    w.a[0] = N->internal ? N->axis : 0;
    w.a[1] = a1;
    w.a[2] = a2;
    for (int ax = 0; ax < 3; ax++) {
        double ext = (double)N->bmax[ax] - (double)N->bmin[ax];
        int e = 1;
        while (e < 254 && 255.0 * ldexp(1.0, e - 127) < ext) e++;
        for (;; e++) {
            if (e > 254) return -1;
            float sc = w_scale(e);
            int ok = isfinite(N->bmin[ax] + 255.0f * sc);
            for (int k = 0; k < 4 && ok; k++) {
                if (slot[k] < 0) continue;
                unsigned lo = 0, hi = 0;
                ok = w_quantize(N->bmin[ax], sc, b->nodes[slot[k]].bmin[ax], b->nodes[slot[k]].bmax[ax], &lo, &hi);
                w.lo[ax][k] = (unsigned char)lo;
                w.hi[ax][k] = (unsigned char)hi;
            }
            if (ok) break;
        }
        w.o[ax] = N->bmin[ax];
        w.s[ax] = w_scale(e);
    }
    for (int k = 0; k < 4; k++) {
        w.child[k] = slot[k];
        w.rec[k] = -1;
    }
    t->r[r] = w;
    for (int k = 0; k < 4; k++) {
        if (slot[k] < 0 || !b->nodes[slot[k]].internal) continue;
        int cr = w_build(b, slot[k], t);
        if (cr < 0) return -1;
        t->r[r].rec[k] = cr;
    }
    return r;
}
/* visit order of the slots (binary near-first DFS): the pair of N's near child first, in a pair
 * its near child first; dsign = ray_dsign with the near flip (1: start is the near child) */
static void w_order(const wrec_t* w, const int* dsign, int* order) {
    int p0 = dsign[w->a[0]] ? 0 : 1;
    for (int q = 0; q < 2; q++) {
        int p = q == 0 ? p0 : 1 - p0;
        int f = dsign[w->a[1 + p]] ? 0 : 1;
        order[2 * q] = 2 * p + f;
        order[2 * q + 1] = 2 * p + 1 - f;
    }
}
static void w_test(const wrec_t* w, const ray3* ray, v3 dinv, int* hit) {
    for (int k = 0; k < 4; k++) {
        hit[k] = 0;
        if (w->child[k] < 0) continue;
        float bmin[3], bmax[3];
        for (int ax = 0; ax < 3; ax++) {  /* byte * scale is exact: one rounding, as the kernel's fma */
            bmin[ax] = w->o[ax] + (float)w->lo[ax][k] * w->s[ax];
            bmax[ax] = w->o[ax] + (float)w->hi[ax][k] * w->s[ax];
        }
        hit[k] = intersect_bbox(ray, dinv, bmin, bmax);
    }
}
static void w_shape(const ctx_t* c, int shape_id, int r, ray3* ray, v3 dinv, const int* dsign, shape_isec* isec,
                    scratch_t* sc) {
    const jt_bvh_tree* bvh = &c->bvh->blas[shape_id];
    const jt_shape* shape = &c->scene->shapes[shape_id];
    const wrec_t* w = &c->wblas[shape_id].r[r];
    sc->cnt.nodes++;
    int hit[4], order[4];
    w_test(w, ray, dinv, hit);
    w_order(w, dsign, order);
    for (int q = 0; q < 4; q++) {
        int k = order[q];
        if (!hit[k]) continue;
        const jt_bvh_node* node = &bvh->nodes[w->child[k]];
        if (node->internal) {
            w_shape(c, shape_id, w->rec[k], ray, dinv, dsign, isec, sc);
            continue;
        }
        for (int i = node->start; i < node->start + node->num; i++) {
            int e = bvh->primitives[i];
            prim_isec p;
            sc->cnt.prims++;
            if (shape->ntriangles > 0) {
                const int32_t* t3 = &shape->triangles[3 * e];
                p = intersect_triangle(ray, pos3(shape, t3[0]), pos3(shape, t3[1]), pos3(shape, t3[2]));
            } else {
                const int32_t* q4 = &shape->quads[4 * e];
                p = intersect_quad(ray, pos3(shape, q4[0]), pos3(shape, q4[1]), pos3(shape, q4[2]), pos3(shape, q4[3]));
            }
            if (!p.hit) continue;
            note_tie(sc, p.distance, ray->tmax);
            isec->element = e;
            isec->uv = p.uv;
            isec->distance = p.distance;
            isec->hit = 1;
            ray->tmax = p.distance;
        }
    }
}
/* intersect_shape_bvh on the wide records */
static shape_isec intersect_shape_wide(const ctx_t* c, int shape_id, ray3 ray, scratch_t* sc, int flip) {
    shape_isec isec = {-1, {0, 0}, 0, 0};
    v3 dinv = V3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    int dsign[3] = {(ray.d.x < 0) ^ flip, (ray.d.y < 0) ^ flip, (ray.d.z < 0) ^ flip};
    w_shape(c, shape_id, 0, &ray, dinv, dsign, &isec, sc);
    return isec;
}
static void w_scene(const ctx_t* c, int r, ray3* ray, v3 dinv, const int* dsign, scene_isec* isec, scratch_t* sc,
                    int flip) {
    const jt_bvh_tree* bvh = &c->bvh->tlas;
    const wrec_t* w = &c->wtlas.r[r];
    sc->cnt.nodes++;
    int hit[4], order[4];
    w_test(w, ray, dinv, hit);
    w_order(w, dsign, order);
    for (int q = 0; q < 4; q++) {
        int k = order[q];
        if (!hit[k]) continue;
        const jt_bvh_node* node = &bvh->nodes[w->child[k]];
        if (node->internal) {
            w_scene(c, w->rec[k], ray, dinv, dsign, isec, sc, flip);
            continue;
        }
        for (int i = node->start; i < node->start + node->num; i++) {
            int inst_id = bvh->primitives[i];
            sc->cnt.instances++;
            ray3 inv_ray = transform_ray(&c->inst_inverse[inst_id], ray);
            shape_isec s = intersect_shape_wide(c, c->scene->instances[inst_id].shape, inv_ray, sc, flip);
            if (!s.hit) continue;
            isec->instance = inst_id;
            isec->element = s.element;
            isec->uv = s.uv;
            isec->distance = s.distance;
            isec->hit = 1;
            ray->tmax = s.distance;
        }
    }
}
/* intersect_scene_bvh on the wide records */
static scene_isec intersect_scene_wide(const ctx_t* c, ray3 ray, scratch_t* sc, int flip) {
    scene_isec isec = {-1, -1, {0, 0}, 0, 0};
    if (c->bvh->tlas.nnodes == 0) return isec;
    v3 dinv = V3(1 / ray.d.x, 1 / ray.d.y, 1 / ray.d.z);
    int dsign[3] = {(ray.d.x < 0) ^ flip, (ray.d.y < 0) ^ flip, (ray.d.z < 0) ^ flip};
    w_scene(c, 0, &ray, dinv, dsign, &isec, sc, flip);
    return isec;
}
/* intersect_instance_bvh on the wide records */
static scene_isec intersect_instance_wide(const ctx_t* c, int inst_id, ray3 ray, scratch_t* sc, int flip) {
    scene_isec isec = {-1, -1, {0, 0}, 0, 0};
    sc->cnt.instances++;
    ray3 inv_ray = transform_ray(&c->inst_inverse[inst_id], &ray);
    shape_isec s = intersect_shape_wide(c, c->scene->instances[inst_id].shape, inv_ray, sc, flip);
    if (!s.hit) return isec;
    isec.instance = inst_id;
    isec.element = s.element;
    isec.uv = s.uv;
    isec.distance = s.distance;
    isec.hit = 1;
    return isec;
}
/* the traversal jt_params.traversal selects; a near-first query that saw an exact-t tie runs again
 * in the reference's child order (the same records) and reports that hit */
static scene_isec scene_query1(const ctx_t* c, ray3 ray, scratch_t* sc) {
    const int wide = c->params->traversal == JT_TRAVERSAL_WIDE, near = c->params->traversal != JT_TRAVERSAL_REFERENCE;
    sc->cnt.rays++;
    sc->tie = 0;
    scene_isec r = wide ? intersect_scene_wide(c, ray, sc, near) : intersect_scene_bvh(c, ray, sc, near);
    if (near && sc->tie) r = wide ? intersect_scene_wide(c, ray, sc, 0) : intersect_scene_bvh(c, ray, sc, 0);
    return r;
}
/* or_order_diff: classify the other order's closest hit against this one's, per query */
static void order_diff(const ctx_t* alt, ray3 ray, scene_isec r, scratch_t* sc) {
    scratch_t tmp = *sc;
    tmp.alt = NULL;
    scene_isec a = scene_query1(alt, ray, &tmp);
    sc->overflow |= tmp.overflow;
    sc->diag[0]++;
    int k;
    if (r.hit != a.hit) k = a.hit ? 3 : 4;                                       /* one order misses */
    else if (!r.hit || (r.instance == a.instance && r.element == a.element)) k = 1; /* same hit */
    else if (r.distance == a.distance) k = 2;                                    /* exact-t tie */
    else k = a.distance < r.distance ? 5 : 6;                                    /* different t */
    sc->diag[k]++;
    if (k != 1) sc->path_diff = 1;
}
static scene_isec scene_query(const ctx_t* c, ray3 ray, scratch_t* sc) {
    scene_isec r = scene_query1(c, ray, sc);
    if (sc->alt) order_diff(sc->alt, ray, r, sc);
    return r;
}
static scene_isec instance_query(const ctx_t* c, int inst_id, ray3 ray, scratch_t* sc) {
    const int wide = c->params->traversal == JT_TRAVERSAL_WIDE, near = c->params->traversal != JT_TRAVERSAL_REFERENCE;
    sc->cnt.light_queries++;
    sc->tie = 0;
    scene_isec r = wide ? intersect_instance_wide(c, inst_id, ray, sc, near) : intersect_instance_bvh(c, inst_id, ray, sc, near);
    /* a one-leaf shape BVH tests its leaf in the same order in every child order: no re-run */
    const jt_bvh_tree* bt = &c->bvh->blas[c->scene->instances[inst_id].shape];
    if (near && sc->tie && bt->nnodes > 0 && bt->nodes[0].internal)
        r = wide ? intersect_instance_wide(c, inst_id, ray, sc, 0) : intersect_instance_bvh(c, inst_id, ray, sc, 0);
    return r;
}

/* --------------------------------------------------------------- scene.jl evaluation */
typedef struct {
    int type;
    v3 emission, color;
    float opacity, roughness, metallic, ior;
    v3 density, scattering;
    float scanisotropy, trdepth;
} material_point; /* MaterialPoint (src/scene.jl:266-320) */

/* eval_position (src/scene.jl:435-476), triangles / quads */
static v3 eval_position(const ctx_t* c, int inst_id, int element, v2 uv) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    const fr3* f = &c->inst_frame[inst_id];
    if (shape->ntriangles != 0) {
        const int32_t* t = &shape->triangles[3 * element];
        return transform_point(f, interp_tri3(pos3(shape, t[0]), pos3(shape, t[1]), pos3(shape, t[2]), uv));
    } else if (shape->nquads != 0) {
        const int32_t* q = &shape->quads[4 * element];
        return transform_point(f, interp_quad3(pos3(shape, q[0]), pos3(shape, q[1]), pos3(shape, q[2]),
                                               pos3(shape, q[3]), uv));
    }
    return V3(0, 0, 0);
}
/* eval_element_normal (src/scene.jl:578-612) */
static v3 eval_element_normal(const ctx_t* c, int inst_id, int element) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    const fr3* f = &c->inst_frame[inst_id];
    if (shape->ntriangles != 0) {
        const int32_t* t = &shape->triangles[3 * element];
        return transform_normal(f, triangle_normal(pos3(shape, t[0]), pos3(shape, t[1]), pos3(shape, t[2])));
    } else if (shape->nquads != 0) {
        const int32_t* q = &shape->quads[4 * element];
        return transform_normal(f, quad_normal(pos3(shape, q[0]), pos3(shape, q[1]), pos3(shape, q[2]),
                                               pos3(shape, q[3])));
    }
    return V3(0, 0, 0);
}
/* eval_normal (src/scene.jl:525-576) */
static v3 eval_normal(const ctx_t* c, int inst_id, int element, v2 uv) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    const fr3* f = &c->inst_frame[inst_id];
    if (shape->nnormals == 0) return eval_element_normal(c, inst_id, element);
    if (shape->ntriangles != 0) {
        const int32_t* t = &shape->triangles[3 * element];
        return transform_normal(f, normalize3(interp_tri3(nrm3(shape, t[0]), nrm3(shape, t[1]), nrm3(shape, t[2]), uv)));
    } else if (shape->nquads != 0) {
        const int32_t* q = &shape->quads[4 * element];
        return transform_normal(f, normalize3(interp_quad3(nrm3(shape, q[0]), nrm3(shape, q[1]), nrm3(shape, q[2]),
                                                           nrm3(shape, q[3]), uv)));
    }
    return V3(0, 0, 0);
}
/* eval_texcoord (src/scene.jl:753-788) */
static v2 eval_texcoord(const ctx_t* c, int inst_id, int element, v2 uv) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    if (shape->ntexcoords == 0) return uv;
    if (shape->ntriangles != 0) {
        const int32_t* t = &shape->triangles[3 * element];
        return interp_tri2(tc2(shape, t[0]), tc2(shape, t[1]), tc2(shape, t[2]), uv);
    } else if (shape->nquads != 0) {
        const int32_t* q = &shape->quads[4 * element];
        return interp_quad2(tc2(shape, q[0]), tc2(shape, q[1]), tc2(shape, q[2]), tc2(shape, q[3]), uv);
    }
    return V2(0, 0);
}
/* eval_color (src/scene.jl:690-720) */
static v4 eval_color(const ctx_t* c, int inst_id, int element, v2 uv) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    if (shape->ncolors == 0) return V4(1, 1, 1, 1);
    if (shape->ntriangles != 0) {
        const int32_t* t = &shape->triangles[3 * element];
        return interp_tri4(col4(shape, t[0]), col4(shape, t[1]), col4(shape, t[2]), uv);
    } else if (shape->nquads != 0) {
        const int32_t* q = &shape->quads[4 * element];
        return interp_quad4(col4(shape, q[0]), col4(shape, q[1]), col4(shape, q[2]), col4(shape, q[3]), uv);
    }
    return V4(0, 0, 0, 0);
}
/* lookup_texture (src/scene.jl:836-849), byte_to_float / srgb_to_rgb (src/color.jl:12-23) */
static v4 lookup_texture(const jt_texture* t, long i, long j, int as_linear) {
    v4 color;
    long k = j * t->width + i;
    if (t->pixelsf) {
        color = V4(t->pixelsf[4 * k], t->pixelsf[4 * k + 1], t->pixelsf[4 * k + 2], t->pixelsf[4 * k + 3]);
    } else {
        const uint8_t* b = &t->pixelsb[4 * k];
        color = V4(b[0] / 255.0f, b[1] / 255.0f, b[2] / 255.0f, b[3] / 255.0f);
    }
    if (as_linear && !t->linear)
        color = V4(srgb_to_rgb1(color.x), srgb_to_rgb1(color.y), srgb_to_rgb1(color.z), color.w);
    return color;
}
/* mod1(x, 1.0f0) for Float32 (base/operators.jl, float.jl: mod via rem) */
static inline float jl_mod1(float x) {
    float r = fmodf(x, 1.0f);
    float m;
    if (r == 0) m = copysignf(r, 1.0f);
    else if ((r > 0) != (1.0f > 0)) m = r + 1.0f;
    else m = r;
    return m == 0 ? 1.0f : m;
}
/* eval_texture (src/scene.jl:790-834), bilinear, wrap */
static v4 eval_texture_t(const jt_texture* t, v2 uv, int as_linear) {
    if (t->width == 0 || t->height == 0) return V4(0, 0, 0, 0);
    long W = t->width, H = t->height;
    float s = jl_mod1(uv.x) * (float)W;
    if (s < 0) s += (float)W;
    float tt = jl_mod1(uv.y) * (float)H;
    if (tt < 0) tt += (float)H;
    long i = jl_clampi((long)truncf(s), 0, W - 1);
    long j = jl_clampi((long)truncf(tt), 0, H - 1);
    long ii = (i + 1) % W, jj = (j + 1) % H;
    float u = s - (float)i, v = tt - (float)j;
    v4 a = scl4(scl4(lookup_texture(t, i, j, as_linear), 1 - u), 1 - v);
    v4 b = scl4(scl4(lookup_texture(t, i, jj, as_linear), 1 - u), v);
    v4 cc = scl4(scl4(lookup_texture(t, ii, j, as_linear), u), 1 - v);
    v4 d = scl4(scl4(lookup_texture(t, ii, jj, as_linear), u), v);
    return add4(add4(add4(a, b), cc), d);
}
static v4 eval_texture(const ctx_t* c, int tex, v2 uv, int as_linear) { /* :675-688 */
    if (tex < 0) return V4(1, 1, 1, 1);
    return eval_texture_t(&c->scene->textures[tex], uv, as_linear);
}
/* eval_element_tangents (src/scene.jl:851-891) */
static void eval_element_tangents(const ctx_t* c, int inst_id, int element, v3* tu, v3* tv) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    const fr3* f = &c->inst_frame[inst_id];
    if (shape->ntriangles != 0 && shape->ntexcoords != 0) {
        const int32_t* t = &shape->triangles[3 * element];
        triangle_tangents_fromuv(pos3(shape, t[0]), pos3(shape, t[1]), pos3(shape, t[2]), tc2(shape, t[0]),
                                 tc2(shape, t[1]), tc2(shape, t[2]), tu, tv);
    } else if (shape->nquads != 0 && shape->ntexcoords != 0) {
        const int32_t* q = &shape->quads[4 * element];
        /* quad_tangents_fromuv with current_uv = (0,0): first triangle (p1,p2,p4) */
        triangle_tangents_fromuv(pos3(shape, q[0]), pos3(shape, q[1]), pos3(shape, q[3]), tc2(shape, q[0]),
                                 tc2(shape, q[1]), tc2(shape, q[3]), tu, tv);
    } else {
        *tu = V3(0, 0, 0);
        *tv = V3(0, 0, 0);
        return;
    }
    *tu = transform_direction(f, *tu);
    *tv = transform_direction(f, *tv);
}
/* eval_normalmap (src/scene.jl:722-751) */
static v3 eval_normalmap(const ctx_t* c, int inst_id, int element, v2 uv) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    const jt_material* m = &c->scene->materials[inst->material];
    v3 normal = eval_normal(c, inst_id, element, uv);
    v2 texcoord = eval_texcoord(c, inst_id, element, uv);
    if (m->normal_tex >= 0 && (shape->ntriangles != 0 || shape->nquads != 0)) {
        v4 t4 = eval_texture_t(&c->scene->textures[m->normal_tex], texcoord, 0);
        v3 nm = V3(t4.x * 2 - 1, t4.y * 2 - 1, t4.z * 2 - 1);
        v3 tu, tv;
        eval_element_tangents(c, inst_id, element, &tu, &tv);
        /* frame = (tu, tv, normal); f1 = orthonormalize(tu, normal); f2 = normalize(cross(normal, tu)) */
        v3 f1 = normalize3(sub3(tu, scl3(normal, dot3(tu, normal))));
        v3 f2 = normalize3(cross3(normal, tu));
        int flip_v = dot3(f2, tv) < 0;
        float n2 = nm.y * (flip_v ? 1.0f : -1.0f);
        nm = V3(nm.x, n2, nm.z);
        fr3 fr;
        fr.x = f1;
        fr.y = f2;
        fr.z = normal;
        fr.o = V3(0, 0, 0);
        normal = transform_normal(&fr, nm);
    }
    return normal;
}
/* eval_shading_normal (src/scene.jl:479-523) */
static v3 eval_shading_normal(const ctx_t* c, int inst_id, int element, v2 uv, v3 outgoing) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_shape* shape = &c->scene->shapes[inst->shape];
    const jt_material* m = &c->scene->materials[inst->material];
    if (shape->ntriangles != 0 || shape->nquads != 0) {
        v3 normal = eval_normal(c, inst_id, element, uv);
        if (m->normal_tex >= 0) normal = eval_normalmap(c, inst_id, element, uv);
        if (m->type == JT_REFRACTIVE) return normal;
        return dot3(normal, outgoing) >= 0 ? normal : neg3(normal);
    }
    return V3(0, 0, 0);
}
/* eval_material (src/scene.jl:615-673) */
static material_point eval_material(const ctx_t* c, int inst_id, int element, v2 uv) {
    const jt_instance* inst = &c->scene->instances[inst_id];
    const jt_material* m = &c->scene->materials[inst->material];
    v2 texcoord = eval_texcoord(c, inst_id, element, uv);
    v4 emission_tex = eval_texture(c, m->emission_tex, texcoord, 1);
    v4 color_shp = eval_color(c, inst_id, element, uv);
    v4 color_tex = eval_texture(c, m->color_tex, texcoord, 1);
    v4 roughness_tex = eval_texture(c, m->roughness_tex, texcoord, 0);
    v4 scattering_tex = eval_texture(c, m->scattering_tex, texcoord, 1);
    material_point p;
    p.type = m->type;
    p.emission = mul3(V3(m->emission[0], m->emission[1], m->emission[2]), xyz(emission_tex));
    p.color = mul3(mul3(V3(m->color[0], m->color[1], m->color[2]), xyz(color_tex)), xyz(color_shp));
    p.opacity = m->opacity * color_tex.w * color_shp.w;
    p.metallic = m->metallic * roughness_tex.z;
    float roughness = m->roughness * roughness_tex.y;
    roughness = roughness * roughness;
    p.ior = m->ior;
    p.scattering = mul3(V3(m->scattering[0], m->scattering[1], m->scattering[2]), xyz(scattering_tex));
    p.scanisotropy = m->scanisotropy;
    p.trdepth = m->trdepth;
    if (m->type == JT_REFRACTIVE || m->type == JT_VOLUMETRIC || m->type == JT_SUBSURFACE) {
        v3 cl = V3(jl_clamp(p.color.x, 0.0001f, 1.0f), jl_clamp(p.color.y, 0.0001f, 1.0f),
                   jl_clamp(p.color.z, 0.0001f, 1.0f));
        p.density = V3(-jl_log(cl.x) / p.trdepth, -jl_log(cl.y) / p.trdepth, -jl_log(cl.z) / p.trdepth);
    } else {
        p.density = V3(0, 0, 0);
    }
    if (p.type == JT_MATTE || p.type == JT_GLTFPBR || p.type == JT_GLOSSY) {
        roughness = jl_clamp(roughness, min_roughness, 1.0f);
    } else if (m->type == JT_VOLUMETRIC) {
        roughness = 0.0f;
    } else if (roughness < min_roughness) {
        roughness = 0.0f;
    }
    p.roughness = roughness;
    return p;
}
/* eval_environment (src/scene.jl:893-914) */
static v3 eval_environment(const ctx_t* c, v3 direction) {
    v3 emission = V3(0, 0, 0);
    for (int e = 0; e < c->scene->nenvironments; e++) {
        const jt_environment* env = &c->scene->environments[e];
        v3 wl = transform_direction(&c->env_inverse[e], direction);
        v2 tc = V2(jl_atan2(wl.z, wl.x) / (2.0f * pif), jl_acos(jl_clamp(wl.y, -1.0f, 1.0f)) / pif);
        if (tc.x < 0.0f) tc.x = tc.x + 1.0f;
        v4 t = eval_texture(c, env->emission_tex, tc, 0);
        v3 em = mul3(V3(env->emission[0], env->emission[1], env->emission[2]), xyz(t));
        emission = add3(emission, em);
    }
    return emission;
}
/* is_delta (src/scene.jl:916-920) */
static inline int is_delta(const material_point* m) {
    return (m->type == JT_REFLECTIVE && m->roughness == 0) || (m->type == JT_REFRACTIVE && m->roughness == 0) ||
           (m->type == JT_TRANSPARENT && m->roughness == 0) || (m->type == JT_VOLUMETRIC);
}
/* is_volumetric(scene, instance) (src/scene.jl:922-928) */
static inline int is_volumetric_inst(const ctx_t* c, int inst_id) {
    int t = c->scene->materials[c->scene->instances[inst_id].material].type;
    return t == JT_REFRACTIVE || t == JT_VOLUMETRIC || t == JT_SUBSURFACE;
}

/* --------------------------------------------------------------- shading.jl */
static inline v3 upn(v3 normal, v3 outgoing) { return dot3(normal, outgoing) <= 0 ? neg3(normal) : normal; }

/* fresnel_dielectric (src/shading.jl:695-714) */
static float fresnel_dielectric(float eta, v3 normal, v3 outgoing) {
    float cosw = fabsf(dot3(normal, outgoing));
    float sin2 = 1 - cosw * cosw;
    float eta2 = eta * eta;
    float cos2t = 1 - sin2 / eta2;
    if (cos2t < 0) return 1;
    float t0 = sqrtf(cos2t);
    float t1 = eta * t0;
    float t2 = eta * cosw;
    float rs = (cosw - t1) / (cosw + t1);
    float rp = (t0 - t2) / (t0 + t2);
    return (rs * rs + rp * rp) / 2;
}
/* fresnel_conductor (src/shading.jl:831-851) */
static float fresnel_conductor1(float eta, float etak, float cosw, float cos2, float sin2) {
    float eta2 = eta * eta, etak2 = etak * etak;
    float t0 = (eta2 - etak2) - sin2;
    float a2plusb2 = sqrtf(t0 * t0 + (4 * eta2) * etak2);
    float t1 = a2plusb2 + cos2;
    float a = sqrtf((a2plusb2 + t0) / 2);
    float t2 = (2 * a) * cosw;
    float rs = (t1 - t2) / (t1 + t2);
    float t3 = cos2 * a2plusb2 + sin2 * sin2;
    float t4 = t2 * sin2;
    float rp = rs * (t3 - t4) / (t3 + t4);
    return (rp + rs) / 2;
}
static v3 fresnel_conductor(v3 eta, v3 etak, v3 normal, v3 outgoing) {
    float cosw = dot3(normal, outgoing);
    if (cosw <= 0) return V3(0, 0, 0);
    cosw = jl_clamp(cosw, -1.0f, 1.0f);
    float cos2 = cosw * cosw;
    float sin2 = jl_clamp(1 - cos2, 0.0f, 1.0f);
    return V3(fresnel_conductor1(eta.x, etak.x, cosw, cos2, sin2), fresnel_conductor1(eta.y, etak.y, cosw, cos2, sin2),
              fresnel_conductor1(eta.z, etak.z, cosw, cos2, sin2));
}
/* reflectivity_to_eta (src/shading.jl:820-823) */
static v3 reflectivity_to_eta(v3 r) {
    v3 c = V3(jl_clamp(r.x, 0.0f, 0.99f), jl_clamp(r.y, 0.0f, 0.99f), jl_clamp(r.z, 0.0f, 0.99f));
    return V3((1 + sqrtf(c.x)) / (1 - sqrtf(c.x)), (1 + sqrtf(c.y)) / (1 - sqrtf(c.y)),
              (1 + sqrtf(c.z)) / (1 - sqrtf(c.z)));
}
/* basis_fromz (src/shading.jl:724-732) */
static m3 basis_fromz(v3 v) {
    v3 z = normalize3(v);
    float sign = copysignf(1.0f, z.z);
    float a = -1.0f / (sign + z.z);
    float b = z.x * z.y * a;
    m3 m;
    m.c1 = V3(1.0f + sign * z.x * z.x * a, sign * b, -sign * z.x);
    m.c2 = V3(b, sign + z.y * z.y * a, -z.y);
    m.c3 = z;
    return m;
}
/* sample_hemisphere_cos (src/shading.jl:716-722) */
static v3 sample_hemisphere_cos(v3 normal, v2 ruv) {
    float z = sqrtf(ruv.y);
    float r = sqrtf(1 - z * z);
    float phi = 2 * pif * ruv.x;
    v3 local = V3(r * jl_cos(phi), r * jl_sin(phi), z);
    m3 b = basis_fromz(normal);
    return m3_transform_direction(&b, local);
}
/* microfacet_distribution, GGX (src/shading.jl:734-750) */
static float microfacet_distribution(float roughness, v3 normal, v3 halfway) {
    float cosine = dot3(normal, halfway);
    if (cosine <= 0) return 0;
    float r2 = roughness * roughness;
    float c2 = cosine * cosine;
    return r2 / (pif * (c2 * r2 + 1 - c2) * (c2 * r2 + 1 - c2));
}
/* microfacet_shadowing1 / microfacet_shadowing (src/shading.jl:752-785) */
static float microfacet_shadowing1(float roughness, v3 normal, v3 halfway, v3 direction) {
    float cosine = dot3(normal, direction);
    float cosineh = dot3(halfway, direction);
    if (cosine * cosineh <= 0) return 0;
    float r2 = roughness * roughness;
    float c2 = cosine * cosine;
    return 2 * fabsf(cosine) / (fabsf(cosine) + sqrtf(c2 - r2 * c2 + r2));
}
static float microfacet_shadowing(float roughness, v3 normal, v3 halfway, v3 outgoing, v3 incoming) {
    return microfacet_shadowing1(roughness, normal, halfway, outgoing) *
           microfacet_shadowing1(roughness, normal, halfway, incoming);
}
/* sample_microfacet, GGX (src/shading.jl:787-803) */
static v3 sample_microfacet(float roughness, v3 normal, v2 rn) {
    float phi = 2 * pif * rn.x;
    float theta = jl_atan(roughness * sqrtf(rn.y / (1 - rn.y)));
    v3 local = V3(jl_cos(phi) * jl_sin(theta), jl_sin(phi) * jl_sin(theta), jl_cos(theta));
    m3 b = basis_fromz(normal);
    return m3_transform_direction(&b, local);
}
/* sample_microfacet_pdf (src/shading.jl:805-816) */
static float sample_microfacet_pdf(float roughness, v3 normal, v3 halfway) {
    float cosine = dot3(normal, halfway);
    if (cosine < 0) return 0;
    return microfacet_distribution(roughness, normal, halfway) * cosine;
}
static inline int same_hemisphere(v3 normal, v3 outgoing, v3 incoming) { /* :828 */
    return dot3(normal, outgoing) * dot3(normal, incoming) >= 0;
}

/* matte (src/shading.jl:14-37) */
static v3 eval_matte(v3 color, v3 normal, v3 outgoing, v3 incoming) {
    if (dot3(normal, incoming) * dot3(normal, outgoing) <= 0) return V3(0, 0, 0);
    return scl3(div3s(color, pif), fabsf(dot3(normal, incoming)));
}
static v3 sample_matte(v3 color, v3 normal, v3 outgoing, v2 rn) {
    (void)color;
    return sample_hemisphere_cos(upn(normal, outgoing), rn);
}
static float sample_matte_pdf(v3 color, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    if (dot3(normal, incoming) * dot3(normal, outgoing) <= 0) return 0;
    return sample_hemisphere_cos_pdf(upn(normal, outgoing), incoming);
}
/* glossy (src/shading.jl:39-101) */
static v3 eval_glossy(v3 color, float ior, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    if (dot3(normal, incoming) * dot3(normal, outgoing) <= 0) return V3(0, 0, 0);
    v3 up = upn(normal, outgoing);
    float F1 = fresnel_dielectric(ior, up, outgoing);
    v3 halfway = normalize3(add3(incoming, outgoing));
    float F = fresnel_dielectric(ior, halfway, incoming);
    float D = microfacet_distribution(roughness, up, halfway);
    float G = microfacet_shadowing(roughness, up, halfway, outgoing, incoming);
    float ci = fabsf(dot3(up, incoming));
    v3 diff = scl3(div3s(scl3(color, 1 - F1), pif), ci);
    float spec = F * D * G / (4 * dot3(up, outgoing) * dot3(up, incoming)) * ci;
    return add3(diff, V3(spec, spec, spec));
}
static v3 sample_glossy(v3 color, float ior, float roughness, v3 normal, v3 outgoing, float rnl, v2 rn) {
    (void)color;
    v3 up = upn(normal, outgoing);
    if (rnl < fresnel_dielectric(ior, up, outgoing)) {
        v3 halfway = sample_microfacet(roughness, up, rn);
        v3 incoming = reflect3(outgoing, halfway);
        if (!same_hemisphere(up, outgoing, incoming)) return V3(0, 0, 0);
        return incoming;
    }
    return sample_hemisphere_cos(up, rn);
}
static float sample_glossy_pdf(v3 color, float ior, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    if (dot3(normal, incoming) * dot3(normal, outgoing) <= 0) return 0;
    v3 up = upn(normal, outgoing);
    v3 halfway = normalize3(add3(outgoing, incoming));
    float F = fresnel_dielectric(ior, up, outgoing);
    return F * sample_microfacet_pdf(roughness, up, halfway) / (4 * fabsf(dot3(outgoing, halfway))) +
           (1 - F) * sample_hemisphere_cos_pdf(up, incoming);
}
/* reflective, rough (src/shading.jl:103-151) */
static v3 eval_reflective_rough(v3 color, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    if (dot3(normal, incoming) * dot3(normal, outgoing) <= 0) return V3(0, 0, 0);
    v3 up = upn(normal, outgoing);
    v3 halfway = normalize3(add3(incoming, outgoing));
    v3 F = fresnel_conductor(reflectivity_to_eta(color), V3(0, 0, 0), halfway, incoming);
    float D = microfacet_distribution(roughness, up, halfway);
    float G = microfacet_shadowing(roughness, up, halfway, outgoing, incoming);
    float den = 4 * dot3(up, outgoing) * dot3(up, incoming);
    float ci = fabsf(dot3(up, incoming));
    return V3(F.x * D * G / den * ci, F.y * D * G / den * ci, F.z * D * G / den * ci);
}
static v3 sample_reflective_rough(v3 color, float roughness, v3 normal, v3 outgoing, v2 rn) {
    (void)color;
    v3 up = upn(normal, outgoing);
    v3 halfway = sample_microfacet(roughness, up, rn);
    v3 incoming = reflect3(outgoing, halfway);
    if (!same_hemisphere(up, outgoing, incoming)) return V3(0, 0, 0);
    return incoming;
}
static float sample_reflective_rough_pdf(v3 color, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    if (dot3(normal, incoming) * dot3(normal, outgoing) <= 0) return 0;
    v3 up = upn(normal, outgoing);
    v3 halfway = normalize3(add3(outgoing, incoming));
    return sample_microfacet_pdf(roughness, up, halfway) / (4 * fabsf(dot3(outgoing, halfway)));
}
/* reflective, delta (src/shading.jl:202-225) */
static v3 eval_reflective_delta(v3 color, v3 normal, v3 outgoing, v3 incoming) {
    if (dot3(normal, incoming) * dot3(normal, outgoing) <= 0) return V3(0, 0, 0);
    v3 up = upn(normal, outgoing);
    return fresnel_conductor(reflectivity_to_eta(color), V3(0, 0, 0), up, outgoing);
}
static v3 sample_reflective_delta(v3 color, v3 normal, v3 outgoing) {
    (void)color;
    return reflect3(outgoing, upn(normal, outgoing));
}
static float sample_reflective_delta_pdf(v3 color, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    return dot3(normal, incoming) * dot3(normal, outgoing) <= 0 ? 0 : 1;
}
/* transparent, rough (src/shading.jl:323-401) */
static v3 eval_transparent_rough(v3 color, float ior, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    v3 up = upn(normal, outgoing);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) {
        v3 halfway = normalize3(add3(incoming, outgoing));
        float F = fresnel_dielectric(ior, halfway, outgoing);
        float D = microfacet_distribution(roughness, up, halfway);
        float G = microfacet_shadowing(roughness, up, halfway, outgoing, incoming);
        float s = F * D * G / (4 * dot3(up, outgoing) * dot3(up, incoming)) * fabsf(dot3(up, incoming));
        return V3(s, s, s);
    } else {
        v3 reflected = reflect3(neg3(incoming), up);
        v3 halfway = normalize3(add3(reflected, outgoing));
        float F = fresnel_dielectric(ior, halfway, outgoing);
        float D = microfacet_distribution(roughness, up, halfway);
        float G = microfacet_shadowing(roughness, up, halfway, outgoing, reflected);
        float den = 4 * dot3(up, outgoing) * dot3(up, reflected);
        float cr = fabsf(dot3(up, reflected));
        return V3(color.x * (1 - F) * D * G / den * cr, color.y * (1 - F) * D * G / den * cr,
                  color.z * (1 - F) * D * G / den * cr);
    }
}
static v3 sample_transparent_rough(v3 color, float ior, float roughness, v3 normal, v3 outgoing, float rnl, v2 rn) {
    (void)color;
    v3 up = upn(normal, outgoing);
    v3 halfway = sample_microfacet(roughness, up, rn);
    if (rnl < fresnel_dielectric(ior, halfway, outgoing)) {
        v3 incoming = reflect3(outgoing, halfway);
        if (!same_hemisphere(up, outgoing, incoming)) return V3(0, 0, 0);
        return incoming;
    } else {
        v3 reflected = reflect3(outgoing, halfway);
        v3 incoming = neg3(reflect3(reflected, up));
        if (same_hemisphere(up, outgoing, incoming)) return V3(0, 0, 0);
        return incoming;
    }
}
static float sample_transparent_rough_pdf(v3 color, float ior, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    v3 up = upn(normal, outgoing);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) {
        v3 halfway = normalize3(add3(incoming, outgoing));
        return fresnel_dielectric(ior, halfway, outgoing) * sample_microfacet_pdf(roughness, up, halfway) /
               (4 * fabsf(dot3(outgoing, halfway)));
    } else {
        v3 reflected = reflect3(neg3(incoming), up);
        v3 halfway = normalize3(add3(reflected, outgoing));
        float d = (1 - fresnel_dielectric(ior, halfway, outgoing)) * sample_microfacet_pdf(roughness, up, halfway);
        return d / (4 * fabsf(dot3(outgoing, halfway)));
    }
}
/* transparent, delta (src/shading.jl:403-446) */
static v3 eval_transparent_delta(v3 color, float ior, v3 normal, v3 outgoing, v3 incoming) {
    v3 up = upn(normal, outgoing);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) {
        float F = fresnel_dielectric(ior, up, outgoing);
        return V3(F, F, F);
    }
    return scl3(color, 1 - fresnel_dielectric(ior, up, outgoing));
}
static v3 sample_transparent_delta(v3 color, float ior, v3 normal, v3 outgoing, float rnl) {
    (void)color;
    v3 up = upn(normal, outgoing);
    if (rnl < fresnel_dielectric(ior, up, outgoing)) return reflect3(outgoing, up);
    return neg3(outgoing);
}
static float sample_transparent_delta_pdf(v3 color, float ior, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    v3 up = upn(normal, outgoing);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) return fresnel_dielectric(ior, up, outgoing);
    return 1 - fresnel_dielectric(ior, up, outgoing);
}
/* refractive, rough (src/shading.jl:448-534) */
static v3 eval_refractive_rough(v3 color, float ior, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    int entering = dot3(normal, outgoing) >= 0;
    v3 up = entering ? normal : neg3(normal);
    float rel_ior = entering ? ior : (1 / ior);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) {
        v3 halfway = normalize3(add3(incoming, outgoing));
        float F = fresnel_dielectric(rel_ior, halfway, outgoing);
        float D = microfacet_distribution(roughness, up, halfway);
        float G = microfacet_shadowing(roughness, up, halfway, outgoing, incoming);
        float s = F * D * G / fabsf(4 * dot3(normal, outgoing) * dot3(normal, incoming)) *
                  fabsf(dot3(normal, incoming));
        return V3(s, s, s);
    } else {
        v3 halfway = scl3(neg3(normalize3(add3(scl3(incoming, rel_ior), outgoing))), entering ? 1.0f : -1.0f);
        float F = fresnel_dielectric(rel_ior, halfway, outgoing);
        float D = microfacet_distribution(roughness, up, halfway);
        float G = microfacet_shadowing(roughness, up, halfway, outgoing, incoming);
        float a = fabsf((dot3(outgoing, halfway) * dot3(incoming, halfway)) /
                        (dot3(outgoing, normal) * dot3(incoming, normal)));
        float sq = rel_ior * dot3(halfway, incoming) + dot3(halfway, outgoing);
        sq = sq * sq; /* ^2.0f0 */
        float s = a * (1 - F) * D * G / sq * fabsf(dot3(normal, incoming));
        return V3(s, s, s);
    }
}
static v3 sample_refractive_rough(v3 color, float ior, float roughness, v3 normal, v3 outgoing, float rnl, v2 rn) {
    (void)color;
    int entering = dot3(normal, outgoing) >= 0;
    v3 up = entering ? normal : neg3(normal);
    v3 halfway = sample_microfacet(roughness, up, rn);
    if (rnl < fresnel_dielectric(entering ? ior : (1 / ior), halfway, outgoing)) {
        v3 incoming = reflect3(outgoing, halfway);
        if (!same_hemisphere(up, outgoing, incoming)) return V3(0, 0, 0);
        return incoming;
    } else {
        v3 incoming = refract3(outgoing, halfway, entering ? (1 / ior) : ior);
        if (same_hemisphere(up, outgoing, incoming)) return V3(0, 0, 0);
        return incoming;
    }
}
static float sample_refractive_rough_pdf(v3 color, float ior, float roughness, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    int entering = dot3(normal, outgoing) >= 0;
    v3 up = entering ? normal : neg3(normal);
    float rel_ior = entering ? ior : (1 / ior);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) {
        v3 halfway = normalize3(add3(incoming, outgoing));
        return fresnel_dielectric(rel_ior, halfway, outgoing) * sample_microfacet_pdf(roughness, up, halfway) /
               (4 * fabsf(dot3(outgoing, halfway)));
    } else {
        v3 halfway = scl3(neg3(normalize3(add3(scl3(incoming, rel_ior), outgoing))), entering ? 1.0f : -1.0f);
        float sq = rel_ior * dot3(halfway, incoming) + dot3(halfway, outgoing);
        sq = sq * sq;
        return (1 - fresnel_dielectric(rel_ior, halfway, outgoing)) * sample_microfacet_pdf(roughness, up, halfway) *
               fabsf(dot3(halfway, incoming)) / sq;
    }
}
/* refractive, delta (src/shading.jl:536-604) */
static v3 eval_refractive_delta(v3 color, float ior, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    if ((double)fabsf(ior - 1) < 1e-3) {
        return dot3(normal, incoming) * dot3(normal, outgoing) <= 0 ? V3(1, 1, 1) : V3(0, 0, 0);
    }
    int entering = dot3(normal, outgoing) >= 0;
    v3 up = entering ? normal : neg3(normal);
    float rel_ior = entering ? ior : (1 / ior);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) {
        float F = fresnel_dielectric(rel_ior, up, outgoing);
        return V3(F, F, F);
    }
    float s = (1 / (rel_ior * rel_ior)) * (1 - fresnel_dielectric(rel_ior, up, outgoing));
    return V3(s, s, s);
}
static v3 sample_refractive_delta(v3 color, float ior, v3 normal, v3 outgoing, float rnl) {
    (void)color;
    if ((double)fabsf(ior - 1) < 1e-3) return neg3(outgoing);
    int entering = dot3(normal, outgoing) >= 0;
    v3 up = entering ? normal : neg3(normal);
    float rel_ior = entering ? ior : (1 / ior);
    if (rnl < fresnel_dielectric(rel_ior, up, outgoing)) return reflect3(outgoing, up);
    return refract3(outgoing, up, 1 / rel_ior);
}
static float sample_refractive_delta_pdf(v3 color, float ior, v3 normal, v3 outgoing, v3 incoming) {
    (void)color;
    if (fabsf(ior - 1) < 0.001f) return dot3(normal, incoming) * dot3(normal, outgoing) < 0 ? 1.0f : 0.0f;
    int entering = dot3(normal, outgoing) >= 0;
    v3 up = entering ? normal : neg3(normal);
    float rel_ior = entering ? ior : (1 / ior);
    if (dot3(normal, incoming) * dot3(normal, outgoing) >= 0) return fresnel_dielectric(rel_ior, up, outgoing);
    return 1 - fresnel_dielectric(rel_ior, up, outgoing);
}
/* passthrough (src/shading.jl:636-646) */
static v3 eval_passthrough(v3 normal, v3 outgoing, v3 incoming) {
    return dot3(normal, incoming) * dot3(normal, outgoing) >= 0 ? V3(0, 0, 0) : V3(1, 1, 1);
}
static float sample_passthrough_pdf(v3 normal, v3 outgoing, v3 incoming) {
    return dot3(normal, incoming) * dot3(normal, outgoing) >= 0 ? 0 : 1;
}
/* transmittance (src/shading.jl:650-669) */
static v3 eval_transmittance(v3 density, float distance) {
    return V3(jl_exp(-density.x * distance), jl_exp(-density.y * distance), jl_exp(-density.z * distance));
}
static float sample_transmittance(v3 density, float max_distance, float rl, float rd) {
    long channel = jl_clampi((long)truncf(rl * 3), 1, 3); /* reference bias kept: channel 3 unreachable */
    float dc = channel == 1 ? density.x : (channel == 2 ? density.y : density.z);
    float distance = dc == 0 ? INFINITY : -jl_log(1 - rd) / dc;
    return jl_min(distance, max_distance);
}
static float sample_transmittance_pdf(v3 density, float distance, float max_distance) {
    if (distance < max_distance) {
        float s = (density.x * jl_exp(-density.x * distance) + density.y * jl_exp(-density.y * distance)) +
                  density.z * jl_exp(-density.z * distance);
        return s / 3;
    }
    float s = (jl_exp(-density.x * max_distance) + jl_exp(-density.y * max_distance)) + jl_exp(-density.z * max_distance);
    return s / 3;
}
/* phase function (src/shading.jl:671-693) */
static float eval_phasefunction(float anisotropy, v3 outgoing, v3 incoming) {
    float cosine = -dot3(outgoing, incoming);
    float denom = 1 + anisotropy * anisotropy - 2 * anisotropy * cosine;
    return (1 - anisotropy * anisotropy) / (4 * pif * denom * sqrtf(denom));
}
static v3 sample_phasefunction(float anisotropy, v3 outgoing, v2 rn) {
    float cos_theta;
    if (fabsf(anisotropy) < 0.001f) {
        cos_theta = 1 - 2 * rn.y;
    } else {
        float square = (1 - anisotropy * anisotropy) / (1 + anisotropy - 2 * anisotropy * rn.y);
        cos_theta = (1 + anisotropy * anisotropy - square * square) / (2 * anisotropy);
    }
    float sin_theta = sqrtf(jl_max(0.0f, 1 - cos_theta * cos_theta));
    float phi = 2 * pif * rn.x;
    v3 local = V3(sin_theta * jl_cos(phi), sin_theta * jl_sin(phi), cos_theta);
    m3 b = basis_fromz(neg3(outgoing));
    return m3_mul(&b, local);
}

/* --------------------------------------------------------- trace.jl dispatch */
/* eval_bsdfcos (src/trace.jl:692-755) */
static v3 eval_bsdfcos(const material_point* m, v3 n, v3 o, v3 i) {
    if (m->roughness == 0) return V3(0, 0, 0);
    switch (m->type) {
        case JT_MATTE: return eval_matte(m->color, n, o, i);
        case JT_GLOSSY: return eval_glossy(m->color, m->ior, m->roughness, n, o, i);
        case JT_REFLECTIVE: return eval_reflective_rough(m->color, m->roughness, n, o, i);
        case JT_TRANSPARENT: return eval_transparent_rough(m->color, m->ior, m->roughness, n, o, i);
        case JT_REFRACTIVE:
        case JT_SUBSURFACE: return eval_refractive_rough(m->color, m->ior, m->roughness, n, o, i);
        default: return V3(0, 0, 0); /* gltfpbr rejected at setup (broken in the reference) */
    }
}
/* eval_delta (src/trace.jl:757-778) */
static v3 eval_delta(const material_point* m, v3 n, v3 o, v3 i) {
    if (m->roughness != 0) return V3(0, 0, 0);
    switch (m->type) {
        case JT_REFLECTIVE: return eval_reflective_delta(m->color, n, o, i);
        case JT_TRANSPARENT: return eval_transparent_delta(m->color, m->ior, n, o, i);
        case JT_REFRACTIVE: return eval_refractive_delta(m->color, m->ior, n, o, i);
        case JT_VOLUMETRIC: return eval_passthrough(n, o, i);
        default: return V3(0, 0, 0);
    }
}
/* sample_bsdfcos (src/trace.jl:780-849) */
static v3 sample_bsdfcos(const material_point* m, v3 n, v3 o, float rnl, v2 rn) {
    if (m->roughness == 0) return V3(0, 0, 0);
    switch (m->type) {
        case JT_MATTE: return sample_matte(m->color, n, o, rn);
        case JT_GLOSSY: return sample_glossy(m->color, m->ior, m->roughness, n, o, rnl, rn);
        case JT_REFLECTIVE: return sample_reflective_rough(m->color, m->roughness, n, o, rn);
        case JT_TRANSPARENT: return sample_transparent_rough(m->color, m->ior, m->roughness, n, o, rnl, rn);
        case JT_REFRACTIVE:
        case JT_SUBSURFACE: return sample_refractive_rough(m->color, m->ior, m->roughness, n, o, rnl, rn);
        default: return V3(0, 0, 0);
    }
}
/* sample_delta (src/trace.jl:851-872) */
static v3 sample_delta(const material_point* m, v3 n, v3 o, float rnl) {
    if (m->roughness != 0) return V3(0, 0, 0);
    switch (m->type) {
        case JT_REFLECTIVE: return sample_reflective_delta(m->color, n, o);
        case JT_TRANSPARENT: return sample_transparent_delta(m->color, m->ior, n, o, rnl);
        case JT_REFRACTIVE: return sample_refractive_delta(m->color, m->ior, n, o, rnl);
        case JT_VOLUMETRIC: return neg3(o);
        default: return V3(0, 0, 0);
    }
}
/* sample_bsdfcos_pdf (src/trace.jl:874-943) */
static float sample_bsdfcos_pdf(const material_point* m, v3 n, v3 o, v3 i) {
    if (m->roughness == 0) return 0;
    switch (m->type) {
        case JT_MATTE: return sample_matte_pdf(m->color, n, o, i);
        case JT_GLOSSY: return sample_glossy_pdf(m->color, m->ior, m->roughness, n, o, i);
        case JT_REFLECTIVE: return sample_reflective_rough_pdf(m->color, m->roughness, n, o, i);
        case JT_TRANSPARENT: return sample_transparent_rough_pdf(m->color, m->ior, m->roughness, n, o, i);
        case JT_REFRACTIVE:
        case JT_SUBSURFACE: return sample_refractive_rough_pdf(m->color, m->ior, m->roughness, n, o, i);
        default: return 0;
    }
}
/* sample_delta_pdf (src/trace.jl:945-966) */
static float sample_delta_pdf(const material_point* m, v3 n, v3 o, v3 i) {
    if (m->roughness != 0) return 0;
    switch (m->type) {
        case JT_REFLECTIVE: return sample_reflective_delta_pdf(m->color, n, o, i);
        case JT_TRANSPARENT: return sample_transparent_delta_pdf(m->color, m->ior, n, o, i);
        case JT_REFRACTIVE: return sample_refractive_delta_pdf(m->color, m->ior, n, o, i);
        case JT_VOLUMETRIC: return sample_passthrough_pdf(n, o, i);
        default: return 0;
    }
}
/* eval_emission (src/trace.jl:575-580) */
static inline v3 eval_emission(const material_point* m, v3 normal, v3 outgoing) {
    return dot3(normal, outgoing) >= 0 ? m->emission : V3(0, 0, 0);
}
/* ---- environment-light alias tables: the build's `env_alias` option (include/jtrace.h,
 * SURVEY §8(f) rank 3), restated here so that option has a seeded checker. The reference draws an
 * environment texel with sample_discrete = upper_bound over the texel CDF (src/sampling.jl:33-56,
 * src/trace.jl:989); the option draws from the same pmf, p_i = cdf[i] - cdf[i-1]
 * (sample_discrete_pdf, src/sampling.jl:39-40), in O(1) with Vose's alias method:
 *   column    c = clamp(trunc(rel * n), 0, n - 1)             (float product, then truncation)
 *   texel idx = (ruv.x < keep[c] ? c : other[c]) + 1           (1-based, as sample_discrete's)
 * The random numbers are the ones the light branch already draws (Appendix A: rl, rel, ruv.x,
 * ruv.y; an environment sample of the reference never reads ruv), so the RNG stream is unchanged.
 * Which CDFs get a table: environment lights whose CDF has >= 1024 entries, is non-decreasing and
 * ends finite and positive (the others keep upper_bound). Table: probabilities scaled to mean 1 in
 * double, columns paired by two LIFO worklists filled in index order (small: < 1, large: >= 1);
 * leftovers of either list keep their own column with probability 1. */
static int g_env_alias = 0;
void or_set_env_alias(int32_t on) { g_env_alias = on != 0; }

static int alias_wanted(const jt_light* l) {
    if (l->environment < 0 || l->ncdf < 1024) return 0;
    for (int32_t i = 1; i < l->ncdf; i++)
        if (!(l->cdf[i] >= l->cdf[i - 1])) return 0;
    const float last = l->cdf[l->ncdf - 1];
    return last > 0 && isfinite(last);
}
static int build_alias(const float* cdf, int32_t n, float* keep, int32_t* other) {
    double* q = (double*)malloc(sizeof(double) * (size_t)n);
    int32_t* small = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    int32_t* large = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    if (!q || !small || !large) { free(q); free(small); free(large); return JT_ERR_NOMEM; }
    double total = 0;
    for (int32_t i = 0; i < n; i++) {
        double p = (double)cdf[i] - (i > 0 ? (double)cdf[i - 1] : 0.0);
        q[i] = p > 0 ? p : 0.0;
        total += q[i];
    }
    int32_t ns = 0, nl = 0;
    for (int32_t i = 0; i < n; i++) {
        q[i] = total > 0 ? q[i] * (double)n / total : 1.0;
        if (q[i] < 1.0) small[ns++] = i;
        else large[nl++] = i;
    }
    while (ns > 0 && nl > 0) {
        const int32_t a = small[--ns], b = large[nl - 1];
        keep[a] = (float)q[a];
        other[a] = b;
        q[b] -= 1.0 - q[a];
        if (q[b] < 1.0) {
            nl--;
            small[ns++] = b;
        }
    }
    for (int32_t k = 0; k < nl; k++) { keep[large[k]] = 1.0f; other[large[k]] = large[k]; }
    for (int32_t k = 0; k < ns; k++) { keep[small[k]] = 1.0f; other[small[k]] = small[k]; }
    free(q);
    free(small);
    free(large);
    return JT_OK;
}
/* the table of one CDF (tests/test_oracle_kat.py): 0 or a negative jt_status */
int or_alias_table(const float* cdf, int32_t n, float* keep, int32_t* other) {
    if (!cdf || n <= 0 || !keep || !other) return JT_ERR_INVALID;
    return build_alias(cdf, n, keep, other);
}
static long sample_alias(const float* keep, const int32_t* other, long n, float rel, float coin) {
    long col = jl_clampi((long)(rel * (float)n), 0, n - 1);
    return (coin < keep[col] ? col : (long)other[col]) + 1;
}

/* sample_lights (src/trace.jl:968-1008) */
static v3 sample_lights(const ctx_t* c, v3 position, float rl, float rel, v2 ruv) {
    long light_id = sample_uniform(c->lights->nlights, rl);
    const jt_light* light = &c->lights->lights[light_id - 1];
    if (light->instance >= 0) {
        const jt_instance* inst = &c->scene->instances[light->instance];
        const jt_shape* shape = &c->scene->shapes[inst->shape];
        long element = sample_discrete(light->cdf, light->ncdf, rel);
        v2 uv = shape->ntriangles != 0 ? sample_triangle(ruv) : ruv;
        v3 lposition = eval_position(c, light->instance, (int)(element - 1), uv);
        return normalize3(sub3(lposition, position));
    } else if (light->environment >= 0) {
        const jt_environment* env = &c->scene->environments[light->environment];
        const jt_texture* tex = &c->scene->textures[env->emission_tex];
        const long li = light - c->lights->lights;
        long idx = c->alias_keep && c->alias_keep[li]  /* 1-based, used as-is (:990-993) */
                       ? sample_alias(c->alias_keep[li], c->alias_other[li], light->ncdf, rel, ruv.x)
                       : sample_discrete(light->cdf, light->ncdf, rel);
        float u = ((float)(idx % tex->width) + 0.5f) / (float)tex->width;
        float v = (float)((((double)idx / (double)tex->width) + 0.5) / (double)tex->height);
        v3 dir = V3(jl_cos(u * 2 * pif) * jl_sin(v * pif), jl_cos(v * pif), jl_sin(u * 2 * pif) * jl_sin(v * pif));
        return transform_direction(&c->env_frame[light->environment], dir);
    }
    return V3(0, 0, 0);
}
/* sample_lights_pdf (src/trace.jl:1010-1084) */
static float sample_lights_pdf(const ctx_t* c, v3 position, v3 direction, scratch_t* sc) {
    float pdf = 0.0f;
    for (int li = 0; li < c->lights->nlights; li++) {
        const jt_light* light = &c->lights->lights[li];
        if (light->instance >= 0) {
            float lpdf = 0.0f;
            v3 next_position = position;
            for (int bounce = 0; bounce < 100; bounce++) {
                scene_isec isec = instance_query(c, light->instance, make_ray(next_position, direction), sc);
                if (!isec.hit) break;
                v3 lposition = eval_position(c, light->instance, isec.element, isec.uv);
                v3 lnormal = eval_element_normal(c, light->instance, isec.element);
                float area = light->cdf[light->ncdf - 1];
                lpdf += distance_squared(lposition, position) / (fabsf(dot3(lnormal, direction)) * area);
                next_position = add3(lposition, scl3(direction, 0.001f));
            }
            pdf += lpdf;
        } else if (light->environment >= 0) {
            const jt_environment* env = &c->scene->environments[light->environment];
            const jt_texture* tex = &c->scene->textures[env->emission_tex];
            v3 wl = transform_direction(&c->env_inverse[light->environment], direction);
            v2 tc = V2(jl_atan2(wl.z, wl.x) / (2 * pif), jl_acos(jl_clamp(wl.y, -1.0f, 1.0f)) / pif);
            if (tc.x < 0) tc.x = tc.x + 1;
            long i = jl_clampi((long)truncf(tc.x * (float)tex->width), 0, tex->width - 1);
            long j = jl_clampi((long)truncf(tc.y * (float)tex->height), 0, tex->height - 1);
            float prob = sample_discrete_pdf(light->cdf, j * tex->width + i + 1) / light->cdf[light->ncdf - 1];
            float angle = (2 * pif / (float)tex->width) * (pif / (float)tex->height) *
                          jl_sin(pif * ((float)j + 0.5f) / (float)tex->height);
            pdf += prob / angle;
        }
    }
    pdf *= sample_uniform_pdf(c->lights->nlights);
    return pdf;
}
/* eval_scattering / sample_scattering / sample_scattering_pdf (src/trace.jl:1086-1115) */
typedef struct { v3 density, scattering; float scanisotropy; } volume_t;
static v3 eval_scattering(const volume_t* m, v3 outgoing, v3 incoming) {
    if (iszero3(m->density)) return V3(0, 0, 0);
    return scl3(mul3(m->scattering, m->density), eval_phasefunction(m->scanisotropy, outgoing, incoming));
}
static v3 sample_scattering(const volume_t* m, v3 outgoing, float rnl, v2 rn) {
    (void)rnl;
    if (iszero3(m->density)) return V3(0, 0, 0);
    return sample_phasefunction(m->scanisotropy, outgoing, rn);
}
static float sample_scattering_pdf(const volume_t* m, v3 outgoing, v3 incoming) {
    if (iszero3(m->density)) return 0;
    return eval_phasefunction(m->scanisotropy, outgoing, incoming);
}

typedef struct { v3 radiance; int hit; v3 albedo, normal; } path_result;

/* trace_path (src/trace.jl:276-469) */
static path_result trace_path(const ctx_t* c, ray3 ray, rng_t* rng, scratch_t* sc) {
    const jt_params* params = c->params;
    v3 radiance = V3(0, 0, 0), weight = V3(1, 1, 1);
    int cur_volume = 0;
    volume_t volume_stack = {{0, 0, 0}, {0, 0, 0}, 0};
    float max_roughness = 0.0f;
    path_result res = {{0, 0, 0}, 0, {0, 0, 0}, {0, 0, 0}};
    int opbounce = 0;
    int bounce = -1;
    while (bounce < params->bounces) {
        bounce += 1;
        scene_isec isec = scene_query(c, ray, sc);
        if (sc->overflow) break;
        if (!isec.hit) {
            if (bounce > 0 || !params->envhidden) radiance = add3(radiance, mul3(weight, eval_environment(c, ray.d)));
            break;
        }
        int in_volume = 0;
        if (cur_volume != 0) {
            const volume_t* vsdf = &volume_stack;
            float rl = rand1f(rng), rd = rand1f(rng);
            float distance = sample_transmittance(vsdf->density, isec.distance, rl, rd);
            v3 tr = eval_transmittance(vsdf->density, distance);
            float tp = sample_transmittance_pdf(vsdf->density, distance, isec.distance);
            weight = div3s(mul3(weight, tr), tp);
            in_volume = distance < isec.distance;
            isec.distance = distance;
        }
        if (!in_volume) {
            v3 outgoing = neg3(ray.d);
            v3 position = eval_position(c, isec.instance, isec.element, isec.uv);
            v3 normal = eval_shading_normal(c, isec.instance, isec.element, isec.uv, outgoing);
            material_point material = eval_material(c, isec.instance, isec.element, isec.uv);
            sc->cnt.shades++;
            if (params->nocaustics) {
                max_roughness = jl_max(material.roughness, max_roughness);
                material.roughness = max_roughness;
            }
            if (material.opacity < 1 && rand1f(rng) >= material.opacity) {
                if (opbounce > 128) break;
                opbounce += 1;
                ray = make_ray(add3(position, scl3(ray.d, 0.01f)), ray.d);
                bounce -= 1;
                continue;
            }
            if (bounce == 0) {
                res.hit = 1;
                res.albedo = material.color;
                res.normal = normal;
            }
            radiance = add3(radiance, mul3(weight, eval_emission(&material, normal, outgoing)));
            v3 incoming = V3(0, 0, 0);
            if (!is_delta(&material)) {
                if (rand1f(rng) < 0.5f) {
                    float rnl = rand1f(rng);
                    v2 rn = rand2f(rng);
                    incoming = sample_bsdfcos(&material, normal, outgoing, rnl, rn);
                } else {
                    float rl = rand1f(rng), rel = rand1f(rng);
                    v2 ruv = rand2f(rng);
                    incoming = sample_lights(c, position, rl, rel, ruv);
                }
                if (iszero3(incoming)) break;
                v3 f = eval_bsdfcos(&material, normal, outgoing, incoming);
                float pb = sample_bsdfcos_pdf(&material, normal, outgoing, incoming);
                float pl = sample_lights_pdf(c, position, incoming, sc);
                weight = div3s(mul3(weight, f), 0.5f * pb + 0.5f * pl);
            } else {
                float rnl = rand1f(rng);
                incoming = sample_delta(&material, normal, outgoing, rnl);
                v3 f = eval_delta(&material, normal, outgoing, incoming);
                float pd = sample_delta_pdf(&material, normal, outgoing, incoming);
                weight = div3s(mul3(weight, f), pd);
            }
            if (is_volumetric_inst(c, isec.instance) && dot3(normal, outgoing) * dot3(normal, incoming) < 0) {
                if (cur_volume == 0) {
                    material_point vm = eval_material(c, isec.instance, isec.element, isec.uv);
                    cur_volume += 1;
                    volume_stack.density = vm.density;
                    volume_stack.scattering = vm.scattering;
                    volume_stack.scanisotropy = vm.scanisotropy;
                } else {
                    cur_volume -= 1;
                }
            }
            ray = make_ray(position, incoming);
        } else {
            v3 outgoing = neg3(ray.d);
            v3 position = add3(ray.o, scl3(ray.d, isec.distance));
            const volume_t* vsdf = &volume_stack;
            v3 incoming = V3(0, 0, 0);
            if (rand1f(rng) < 0.5f) {
                float rnl = rand1f(rng);
                v2 rn = rand2f(rng);
                incoming = sample_scattering(vsdf, outgoing, rnl, rn);
            } else {
                float rl = rand1f(rng), rel = rand1f(rng);
                v2 ruv = rand2f(rng);
                incoming = sample_lights(c, position, rl, rel, ruv);
            }
            if (iszero3(incoming)) break;
            v3 f = eval_scattering(vsdf, outgoing, incoming);
            float ps = sample_scattering_pdf(vsdf, outgoing, incoming);
            float pl = sample_lights_pdf(c, position, incoming, sc);
            weight = div3s(mul3(weight, f), 0.5f * ps + 0.5f * pl);
            ray = make_ray(position, incoming);
        }
        if (iszero3(weight) || !isfinite3(weight)) break;
        if (bounce > 3) {
            float rr_prob = jl_min(0.99f, max3f(weight));
            if (rand1f(rng) >= rr_prob) break;
            weight = scl3(weight, 1 / rr_prob);
        }
    }
    res.radiance = radiance;
    return res;
}

/* trace_naive (src/trace.jl:471-573) */
static path_result trace_naive(const ctx_t* c, ray3 ray, rng_t* rng, scratch_t* sc) {
    const jt_params* params = c->params;
    v3 radiance = V3(0, 0, 0), weight = V3(1, 1, 1);
    path_result res = {{0, 0, 0}, 0, {0, 0, 0}, {0, 0, 0}};
    int opbounce = 0;
    int bounce = -1;
    while (bounce < params->bounces) {
        bounce += 1;
        scene_isec isec = scene_query(c, ray, sc);
        if (sc->overflow) break;
        if (!isec.hit) {
            if (bounce > 0 || !params->envhidden) radiance = add3(radiance, mul3(weight, eval_environment(c, ray.d)));
            break;
        }
        v3 outgoing = neg3(ray.d);
        v3 position = eval_position(c, isec.instance, isec.element, isec.uv);
        v3 normal = eval_shading_normal(c, isec.instance, isec.element, isec.uv, outgoing);
        material_point material = eval_material(c, isec.instance, isec.element, isec.uv);
        sc->cnt.shades++;
        if (material.opacity < 1 && rand1f(rng) >= material.opacity) {
            if (opbounce > 128) break;
            opbounce += 1;
            ray = make_ray(add3(position, scl3(ray.d, 0.01f)), ray.d);
            bounce -= 1;
            continue;
        }
        if (bounce == 0) {
            res.hit = 1;
            res.albedo = material.color;
            res.normal = normal;
        }
        radiance = add3(radiance, mul3(weight, eval_emission(&material, normal, outgoing)));
        v3 incoming;
        if (material.roughness != 0) {
            float rnl = rand1f(rng);
            v2 rn = rand2f(rng);
            incoming = sample_bsdfcos(&material, normal, outgoing, rnl, rn);
            if (iszero3(incoming)) break;
            v3 f = eval_bsdfcos(&material, normal, outgoing, incoming);
            float p = sample_bsdfcos_pdf(&material, normal, outgoing, incoming);
            weight = div3s(mul3(weight, f), p);
        } else {
            float rnl = rand1f(rng);
            incoming = sample_delta(&material, normal, outgoing, rnl);
            if (iszero3(incoming)) break;
            v3 f = eval_delta(&material, normal, outgoing, incoming);
            float p = sample_delta_pdf(&material, normal, outgoing, incoming);
            weight = div3s(mul3(weight, f), p);
        }
        if (iszero3(weight) || !isfinite3(weight)) break;
        if (bounce > 3) {
            float rr_prob = jl_min(0.99f, max3f(weight));
            if (rand1f(rng) >= rr_prob) break;
            weight = scl3(weight, 1 / rr_prob);
        }
        ray = make_ray(position, incoming);
    }
    res.radiance = radiance;
    return res;
}

/* eval_camera (src/scene.jl:372-411); `aspect` is camera.aspect (:377-378), or W/H under the
 * --width/--height extension (setup_ctx) */
static ray3 eval_camera(const jt_camera* cam, float aspect, const fr3* frame, v2 image_uv, v2 lens_uv) {
    v2 film = aspect >= 1 ? V2(cam->film, cam->film / aspect) : V2(cam->film * aspect, cam->film);
    if (!cam->orthographic) {
        v3 q = V3(film.x * (0.5f - image_uv.x), film.y * (image_uv.y - 0.5f), cam->lens);
        v3 dc = neg3(normalize3(q));
        v3 e = V3(lens_uv.x * cam->aperture / 2, lens_uv.y * cam->aperture / 2, 0);
        v3 p = div3s(scl3(dc, cam->focus), fabsf(dc.z));
        v3 d = normalize3(sub3(p, e));
        return make_ray(transform_point(frame, e), transform_direction(frame, d));
    } else {
        float scale = 1 / cam->lens;
        v3 q = V3(film.x * (0.5f - image_uv.x) * scale, film.y * (image_uv.y - 0.5f) * scale, cam->lens);
        v3 e = add3(V3(-q.x, -q.y, 0), V3(lens_uv.x * cam->aperture / 2, lens_uv.y * cam->aperture / 2, 0));
        v3 p = V3(-q.x, -q.y, -cam->focus);
        v3 d = normalize3(sub3(p, e));
        return make_ray(transform_point(frame, e), transform_direction(frame, d));
    }
}
/* sample_camera (src/trace.jl:651-674) */
static ray3 sample_camera(const ctx_t* c, const jt_camera* cam, int i, int j, v2 puv, v2 luv, int tent) {
    if (!tent) {
        v2 uv = V2(((float)i + puv.x) / (float)c->width, ((float)j + puv.y) / (float)c->height);
        return eval_camera(cam, c->camera_aspect, &c->camera_frame, uv, sample_disk(luv));
    }
    float width = 2.0f, offset = 0.5f;
    v2 fuv = V2(width * (puv.x < 0.5f ? sqrtf(2 * puv.x) - 1 : 1 - sqrtf(2 - 2 * puv.x)) + offset,
                width * (puv.y < 0.5f ? sqrtf(2 * puv.y) - 1 : 1 - sqrtf(2 - 2 * puv.y)) + offset);
    v2 uv = V2(((float)i + fuv.x) / (float)c->width, ((float)j + fuv.y) / (float)c->height);
    return eval_camera(cam, c->camera_aspect, &c->camera_frame, uv, sample_disk(luv));
}

typedef struct {
    const ctx_t* c;
    int32_t first, s0, s1, row0, row1, nthreads, tid, lk;
    float *image, *albedo, *normal;
    int64_t* hits;
    /* the sample streams' running means (lk > 0): stream j of pixel p at [j * W*H + p] */
    float *part_img, *part_alb, *part_nrm;
    int64_t* part_hits;
    scratch_t sc;
} worker_t;

/* trace_sample (src/trace.jl:584-649) for one pixel over [s0, s1).
 * Sample streams (the build's accumulation contract, include/jtrace.h jt_trace_range): local
 * sample t = sample - first belongs to stream t mod 2^lk and is its (t >> lk)-th sample; each
 * stream keeps the reference's running mean of its own samples (src/trace.jl:631-648). lk = 0 is
 * the reference's single running mean over all samples, kept in the image buffers themselves.
 * After the range the streams are combined into the image buffers (combine_pixel). */
static void trace_pixel(worker_t* w, int i, int j) {
    const ctx_t* c = w->c;
    const jt_params* params = c->params;
    const jt_camera* cam = &c->scene->cameras[params->camera];
    long idx = (long)c->width * j + i;
    const long npix = (long)c->width * c->height;
    for (int32_t sample = w->s0; sample < w->s1; sample++) {
        rng_t rng = rng_init(params->seed, (int32_t)idx, sample);
        v2 puv = rand2f(&rng);
        v2 luv = rand2f(&rng);
        ray3 ray = sample_camera(c, cam, i, j, puv, luv, params->tentfilter);
        path_result r;
        if (params->sampler == JT_SAMPLER_NAIVE) r = trace_naive(c, ray, &rng, &w->sc);
        else r = trace_path(c, ray, &rng, &w->sc);
        w->sc.cnt.paths++;
        if (w->sc.path_diff) {
            w->sc.diag[7]++;
            w->sc.path_diff = 0;
        }
        v3 radiance = r.radiance;
        if (!isfinite3(radiance)) radiance = V3(0, 0, 0);
        float mr = max3f(radiance);
        if (mr > (float)params->clamp) radiance = scl3(radiance, (float)params->clamp / mr);
        const int32_t t = sample - w->first;
        const long sidx = w->lk ? (long)(t & ((1 << w->lk) - 1)) * npix + idx : idx;
        float weight = 1.0f / (float)((t >> w->lk) + 1);
        float* im = w->lk ? &w->part_img[4 * sidx] : &w->image[4 * idx];
        float* al = w->lk ? &w->part_alb[3 * sidx] : &w->albedo[3 * idx];
        float* nm = w->lk ? &w->part_nrm[3 * sidx] : &w->normal[3 * idx];
        int64_t* hp = w->lk ? &w->part_hits[sidx] : &w->hits[idx];
        v4 img = V4(im[0], im[1], im[2], im[3]);
        v3 alb = V3(al[0], al[1], al[2]);
        v3 nrm = V3(nm[0], nm[1], nm[2]);
        v4 target4;
        v3 target_a, target_n;
        if (r.hit) {
            target4 = V4(radiance.x, radiance.y, radiance.z, 1);
            target_a = r.albedo;
            target_n = r.normal;
            *hp += 1;
        } else if (!params->envhidden && c->scene->nenvironments != 0) {
            target4 = V4(radiance.x, radiance.y, radiance.z, 1);
            target_a = V3(1, 1, 1);
            target_n = neg3(ray.d);
            *hp += 1;
        } else {
            target4 = V4(0, 0, 0, 0);
            target_a = V3(0, 0, 0);
            target_n = neg3(ray.d);
        }
        /* lerp(a, b, u) = @. a * (1 - u) + b * u (src/math.jl:89-93) */
        float omw = 1 - weight;
        img = add4(scl4(img, omw), scl4(target4, weight));
        alb = add3(scl3(alb, omw), scl3(target_a, weight));
        nrm = add3(scl3(nrm, omw), scl3(target_n, weight));
        im[0] = img.x; im[1] = img.y; im[2] = img.z; im[3] = img.w;
        al[0] = alb.x; al[1] = alb.y; al[2] = alb.z;
        nm[0] = nrm.x; nm[1] = nrm.y; nm[2] = nrm.z;
        if (w->sc.overflow) return;
    }
}

/* the streams' means combined in stream order after the range (include/jtrace.h jt_trace_range):
 * n local samples so far, stream j holds n_j of them, w_j = (float)((double)n_j / n);
 * mean = mean_0 * w_0 + mean_1 * w_1 + ... (no FMA), hits = sum_j hits_j */
static void combine_pixel(worker_t* w, long idx) {
    const long npix = (long)w->c->width * w->c->height;
    const long n = (long)w->s1 - w->first, k = 1L << w->lk;
    const long ns = n < k ? n : k;
    float im[4] = {0, 0, 0, 0}, al[3] = {0, 0, 0}, nm[3] = {0, 0, 0};
    int64_t h = 0;
    for (long s = 0; s < ns; s++) {
        const float ws = (float)((double)((n - 1 - s) / k + 1) / (double)n);
        const long o = s * npix + idx;
        for (int q = 0; q < 4; q++) im[q] = s == 0 ? w->part_img[4 * o + q] * ws : im[q] + w->part_img[4 * o + q] * ws;
        for (int q = 0; q < 3; q++) al[q] = s == 0 ? w->part_alb[3 * o + q] * ws : al[q] + w->part_alb[3 * o + q] * ws;
        for (int q = 0; q < 3; q++) nm[q] = s == 0 ? w->part_nrm[3 * o + q] * ws : nm[q] + w->part_nrm[3 * o + q] * ws;
        h += w->part_hits[o];
    }
    for (int q = 0; q < 4; q++) w->image[4 * idx + q] = im[q];
    for (int q = 0; q < 3; q++) w->albedo[3 * idx + q] = al[q];
    for (int q = 0; q < 3; q++) w->normal[3 * idx + q] = nm[q];
    w->hits[idx] = h;
}

static void* worker_main(void* arg) {
    worker_t* w = (worker_t*)arg;
    for (int j = w->row0 + w->tid; j < w->row1; j += w->nthreads) {
        for (int i = 0; i < w->c->width; i++) {
            trace_pixel(w, i, j);
            if (w->sc.overflow) return NULL;
            if (w->lk) combine_pixel(w, (long)w->c->width * j + i);
        }
    }
    return NULL;
}

static int setup_ctx(ctx_t* c, const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights,
                     const jt_params* params, int width, int height) {
    memset(c, 0, sizeof(*c));
    c->scene = scene;
    c->bvh = bvh;
    c->lights = lights;
    c->params = params;
    c->width = width;
    c->height = height;
    if (params->camera < 0 || params->camera >= scene->ncameras) return JT_ERR_INVALID;
    c->camera_frame = frame_from(scene->cameras[params->camera].frame);
    /* The reference sizes the film from camera.aspect only (src/scene.jl:377-378, src/trace.jl:189-197
     * derives W,H from it). The build's --width/--height extension renders an explicit W x H frame
     * (the 1280x720 headline config of a 1:1 cornellbox camera) and fits the film to it:
     * aspect := W/H (float division), as jt_create does (jt_trace.hip, DParams.cam.aspect). */
    c->camera_aspect = (params->width > 0 && params->height > 0) ? (float)width / (float)height
                                                                 : scene->cameras[params->camera].aspect;
    c->inst_frame = (fr3*)malloc(sizeof(fr3) * (size_t)(scene->ninstances + 1));
    c->inst_inverse = (fr3*)malloc(sizeof(fr3) * (size_t)(scene->ninstances + 1));
    c->env_frame = (fr3*)malloc(sizeof(fr3) * (size_t)(scene->nenvironments + 1));
    c->env_inverse = (fr3*)malloc(sizeof(fr3) * (size_t)(scene->nenvironments + 1));
    if (!c->inst_frame || !c->inst_inverse || !c->env_frame || !c->env_inverse) return JT_ERR_NOMEM;
    for (int k = 0; k < scene->ninstances; k++) {
        c->inst_frame[k] = frame_from(scene->instances[k].frame);
        c->inst_inverse[k] = inverse_frame(&c->inst_frame[k], 1);
    }
    for (int k = 0; k < scene->nenvironments; k++) {
        c->env_frame[k] = frame_from(scene->environments[k].frame);
        c->env_inverse[k] = inverse_frame(&c->env_frame[k], 0);
    }
    if (g_env_alias) {
        c->alias_keep = (float**)calloc((size_t)lights->nlights + 1, sizeof(float*));
        c->alias_other = (int32_t**)calloc((size_t)lights->nlights + 1, sizeof(int32_t*));
        if (!c->alias_keep || !c->alias_other) return JT_ERR_NOMEM;
        for (int k = 0; k < lights->nlights; k++) {
            const jt_light* l = &lights->lights[k];
            if (!alias_wanted(l)) continue;
            c->alias_keep[k] = (float*)malloc(sizeof(float) * (size_t)l->ncdf);
            c->alias_other[k] = (int32_t*)malloc(sizeof(int32_t) * (size_t)l->ncdf);
            if (!c->alias_keep[k] || !c->alias_other[k]) return JT_ERR_NOMEM;
            int st = build_alias(l->cdf, l->ncdf, c->alias_keep[k], c->alias_other[k]);
            if (st != JT_OK) return st;
        }
    }
    if (params->traversal == JT_TRAVERSAL_WIDE) {
        c->wblas = (wtree_t*)calloc((size_t)scene->nshapes + 1, sizeof(wtree_t));
        if (!c->wblas) return JT_ERR_NOMEM;
        if (bvh->tlas.nnodes > 0 && w_build(&bvh->tlas, 0, &c->wtlas) < 0) return JT_ERR_UNSUPPORTED;
        for (int s = 0; s < scene->nshapes; s++)
            if (bvh->blas[s].nnodes > 0 && w_build(&bvh->blas[s], 0, &c->wblas[s]) < 0) return JT_ERR_UNSUPPORTED;
    } else if (params->traversal != JT_TRAVERSAL_REFERENCE && params->traversal != JT_TRAVERSAL_NEAR) {
        return JT_ERR_INVALID;
    }
    return JT_OK;
}
static void free_ctx(ctx_t* c) {
    free(c->inst_frame);
    free(c->inst_inverse);
    free(c->env_frame);
    free(c->env_inverse);
    free(c->wtlas.r);
    if (c->wblas)
        for (int s = 0; s < c->scene->nshapes; s++) free(c->wblas[s].r);
    free(c->wblas);
    if (c->alias_keep)
        for (int k = 0; k < c->lights->nlights; k++) {
            free(c->alias_keep[k]);
            free(c->alias_other[k]);
        }
    free(c->alias_keep);
    free(c->alias_other);
}

static int trace_rows_impl(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights,
                           const jt_params* params, int32_t width, int32_t height, int32_t row0, int32_t row1,
                           int32_t first, int32_t s0, int32_t s1, float* image, float* albedo, float* normal,
                           int64_t* hits, int32_t lk, float* part_img, float* part_alb, float* part_nrm,
                           int64_t* part_hits, int32_t nthreads, or_counters* counters, const jt_params* alt_params,
                           uint64_t* diag);
int or_trace_rows(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights, const jt_params* params,
                  int32_t width, int32_t height, int32_t row0, int32_t row1, int32_t first, int32_t s0, int32_t s1,
                  float* image, float* albedo, float* normal, int64_t* hits, int32_t lk, float* part_img,
                  float* part_alb, float* part_nrm, int64_t* part_hits, int32_t nthreads, or_counters* counters) {
    return trace_rows_impl(scene, bvh, lights, params, width, height, row0, row1, first, s0, s1, image, albedo, normal,
                           hits, lk, part_img, part_alb, part_nrm, part_hits, nthreads, counters, NULL, NULL);
}

/* Diagnostic (tests/test_oracle_traversal.py): trace samples [s0, s1) of every pixel in
 * params->traversal and, at every closest-hit scene query, also run the query in alt_traversal
 * on the same ray. diag[0] queries, [1] same hit, [2] another primitive at exactly the same t,
 * [3] only the alternative order hits, [4] only this order hits, [5] the alternative's hit is
 * closer, [6] farther, [7] paths with at least one differing query. */
int or_order_diff(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights, const jt_params* params,
                  int32_t alt_traversal, int32_t width, int32_t height, int32_t s0, int32_t s1, int32_t nthreads,
                  uint64_t* diag) {
    jt_params alt = *params;
    alt.traversal = alt_traversal;
    size_t np = (size_t)width * height;
    float* im = (float*)calloc(np * 4, sizeof(float));
    float* al = (float*)calloc(np * 3, sizeof(float));
    float* nm = (float*)calloc(np * 3, sizeof(float));
    int64_t* h = (int64_t*)calloc(np, sizeof(int64_t));
    int st = (im && al && nm && h) ? trace_rows_impl(scene, bvh, lights, params, width, height, 0, height, s0, s0, s1, im, al,
                                                     nm, h, 0, NULL, NULL, NULL, NULL, nthreads, NULL, &alt, diag)
                                   : JT_ERR_NOMEM;
    free(im);
    free(al);
    free(nm);
    free(h);
    return st;
}

static int trace_rows_impl(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights,
                           const jt_params* params, int32_t width, int32_t height, int32_t row0, int32_t row1,
                           int32_t first, int32_t s0, int32_t s1, float* image, float* albedo, float* normal,
                           int64_t* hits, int32_t lk, float* part_img, float* part_alb, float* part_nrm,
                           int64_t* part_hits, int32_t nthreads, or_counters* counters, const jt_params* alt_params,
                           uint64_t* diag) {
    if (!scene || !bvh || !lights || !params || !image || !albedo || !normal || !hits) return JT_ERR_INVALID;
    if (lk < 0 || lk > 6 || (lk > 0 && (!part_img || !part_alb || !part_nrm || !part_hits))) return JT_ERR_INVALID;
    if (width <= 0 || height <= 0 || s0 < first || s1 < s0 || row0 < 0 || row1 > height) return JT_ERR_INVALID;
    if (nthreads < 1) nthreads = 1;
    ctx_t c, alt;
    int st = setup_ctx(&c, scene, bvh, lights, params, width, height);
    if (st != JT_OK) { free_ctx(&c); return st; }
    if (alt_params) {
        st = setup_ctx(&alt, scene, bvh, lights, alt_params, width, height);
        if (st != JT_OK) { free_ctx(&alt); free_ctx(&c); return st; }
    }
    worker_t* ws = (worker_t*)calloc((size_t)nthreads, sizeof(worker_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    int ssize = params->bvhstacksize > 0 ? params->bvhstacksize : 128;
    for (int t = 0; t < nthreads; t++) {
        worker_t* w = &ws[t];
        w->c = &c;
        w->first = first;
        w->s0 = s0;
        w->s1 = s1;
        w->row0 = row0;
        w->row1 = row1;
        w->nthreads = nthreads;
        w->tid = t;
        w->image = image;
        w->albedo = albedo;
        w->normal = normal;
        w->hits = hits;
        w->lk = lk;
        w->part_img = part_img;
        w->part_alb = part_alb;
        w->part_nrm = part_nrm;
        w->part_hits = part_hits;
        w->sc.alt = alt_params ? &alt : NULL;
        w->sc.stack = (int32_t*)malloc(sizeof(int32_t) * (size_t)ssize);
        w->sc.sub_stack = (int32_t*)malloc(sizeof(int32_t) * (size_t)ssize);
        w->sc.stack_size = ssize;
    }
    if (nthreads == 1) {
        worker_main(&ws[0]);
    } else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker_main, &ws[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    int overflow = 0;
    or_counters total = {0, 0, 0, 0, 0, 0, 0};
    for (int t = 0; t < nthreads; t++) {
        worker_t* w = &ws[t];
        overflow |= w->sc.overflow;
        total.paths += w->sc.cnt.paths;
        total.rays += w->sc.cnt.rays;
        total.light_queries += w->sc.cnt.light_queries;
        total.nodes += w->sc.cnt.nodes;
        total.instances += w->sc.cnt.instances;
        total.prims += w->sc.cnt.prims;
        total.shades += w->sc.cnt.shades;
        if (diag)
            for (int k = 0; k < 10; k++) diag[k] += w->sc.diag[k];
        free(w->sc.stack);
        free(w->sc.sub_stack);
    }
    if (counters) *counters = total;
    free(ws);
    free(th);
    free_ctx(&c);
    if (alt_params) free_ctx(&alt);
    return overflow ? JT_ERR_STACK : JT_OK;
}

int or_trace(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights, const jt_params* params,
             int32_t width, int32_t height, int32_t first, int32_t s0, int32_t s1, float* image, float* albedo,
             float* normal, int64_t* hits, int32_t nthreads, or_counters* counters) {
    return or_trace_rows(scene, bvh, lights, params, width, height, 0, height, first, s0, s1, image, albedo, normal,
                         hits, 0, NULL, NULL, NULL, NULL, nthreads, counters);
}

/* ================================================================ BVH build (src/bvh.jl) */
typedef struct { v3 min, max; } bbox3;
static inline bbox3 bbox_empty(void) { /* Bbox3f() (src/geometry.jl:26-29) */
    bbox3 b = {{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
    return b;
}
static inline bbox3 merge_pt(bbox3 b, v3 p) { /* merge_bbox3f (:88-89) */
    bbox3 r = {{jl_min(b.min.x, p.x), jl_min(b.min.y, p.y), jl_min(b.min.z, p.z)},
               {jl_max(b.max.x, p.x), jl_max(b.max.y, p.y), jl_max(b.max.z, p.z)}};
    return r;
}
static inline bbox3 merge_bb(bbox3 a, bbox3 b) { /* :91-92 */
    bbox3 r = {{jl_min(a.min.x, b.min.x), jl_min(a.min.y, b.min.y), jl_min(a.min.z, b.min.z)},
               {jl_max(a.max.x, b.max.x), jl_max(a.max.y, b.max.y), jl_max(a.max.z, b.max.z)}};
    return r;
}
static inline v3 bbox_center(bbox3 b) { return div3s(add3(b.min, b.max), 2); } /* :94 */
static inline float comp(v3 v, int axis1) { return axis1 == 1 ? v.x : (axis1 == 2 ? v.y : v.z); }
static float bbox_area(bbox3 b) { /* src/bvh.jl:276-279 */
    v3 s = sub3(b.max, b.min);
    return 0.000000000001f + 2 * s.x * s.y + 2 * s.x * s.z + 2 * s.y * s.z;
}
/* partition (src/bvh.jl:281-304); prims 1-based array view */
static long partition(const v3* centers, int axis, float split, long* prims, long start, long stop) {
    long i = start, j = stop;
    while (1) {
        while (i <= stop && comp(centers[prims[i]], axis) < split) i += 1;
        while (j >= start && comp(centers[prims[j]], axis) >= split) j -= 1;
        if (i >= j) break;
        long tmp = prims[i];
        prims[i] = prims[j];
        prims[j] = tmp;
    }
    return j;
}
/* split_middle (src/bvh.jl:185-216) */
static void split_middle(long* prims, const v3* centers, long left, long right, long* mid, int* axis_out) {
    bbox3 cb = bbox_empty();
    for (long i = left; i <= right; i++) cb = merge_pt(cb, centers[prims[i]]);
    v3 cs = sub3(cb.max, cb.min);
    if (cs.x == 0 && cs.y == 0 && cs.z == 0) { *mid = (left + right + 1) / 2; *axis_out = 1; return; }
    int axis = 1;
    if (cs.x >= cs.y && cs.x >= cs.z) axis = 1;
    if (cs.y >= cs.x && cs.y >= cs.z) axis = 2;
    if (cs.z >= cs.x && cs.z >= cs.y) axis = 3;
    float split = comp(bbox_center(cb), axis);
    long middle = partition(centers, axis, split, prims, left, right);
    if (middle < left || middle > right) { *mid = (left + right + 1) / 2; *axis_out = axis; return; }
    *mid = middle;
    *axis_out = axis;
}
/* split_sah (src/bvh.jl:218-274) */
static void split_sah(long* prims, const bbox3* bboxes, const v3* centers, long left, long right, long* mid,
                      int* axis_out) {
    bbox3 cb = bbox_empty();
    for (long i = left; i <= right; i++) cb = merge_pt(cb, centers[prims[i]]);
    v3 cs = sub3(cb.max, cb.min);
    if (cs.x == 0 && cs.y == 0 && cs.z == 0) { *mid = (left + right + 1) / 2; *axis_out = 1; return; }
    int axis = 1;
    const int nbins = 16;
    float split = 0.0f;
    float min_cost = INFINITY;
    for (int saxis = 1; saxis <= 3; saxis++) {
        for (int b = 1; b <= nbins - 1; b++) {
            float bsplit = comp(cb.min, saxis) + (float)b * comp(cs, saxis) / (float)nbins;
            bbox3 lb = bbox_empty(), rb = bbox_empty();
            long ln = 0, rn = 0;
            for (long i = left; i <= right; i++) {
                if (comp(centers[prims[i]], saxis) < bsplit) { lb = merge_bb(lb, bboxes[prims[i]]); ln++; }
                else { rb = merge_bb(rb, bboxes[prims[i]]); rn++; }
            }
            float cost = 1 + (float)ln * bbox_area(lb) / bbox_area(cb) + (float)rn * bbox_area(rb) / bbox_area(cb);
            if (cost < min_cost) { min_cost = cost; split = bsplit; axis = saxis; }
        }
    }
    long middle = partition(centers, axis, split, prims, left, right);
    if (middle == left || middle == right) { *mid = (left + right + 1) / 2; *axis_out = axis; return; }
    *mid = middle;
    *axis_out = axis;
}
/* make_bvh (src/bvh.jl:138-183); bboxes 1-based (index 0 unused) */
static int make_bvh(const bbox3* bboxes, long n, int hq, jt_bvh_tree* out) {
    long cap = 2 * n + 2;
    jt_bvh_node* nodes = (jt_bvh_node*)calloc((size_t)cap, sizeof(jt_bvh_node));
    long* prims = (long*)malloc(sizeof(long) * (size_t)(n + 1));
    v3* centers = (v3*)malloc(sizeof(v3) * (size_t)(n + 1));
    long* stk = (long*)malloc(sizeof(long) * 3 * (size_t)(cap + 1));
    bbox3* nb = (bbox3*)malloc(sizeof(bbox3) * (size_t)cap);
    if (!nodes || !prims || !centers || !stk || !nb) return JT_ERR_NOMEM;
    for (long i = 1; i <= n; i++) { prims[i] = i; centers[i] = bbox_center(bboxes[i]); }
    long nnodes = 0;
    long sp = 0;
    stk[0] = 1; stk[1] = 1; stk[2] = n; sp = 1;
    nnodes = 1; /* push!(bvh.nodes, BvhNode()) */
    nb[0] = bbox_empty();
    nodes[0].axis = 0;
    while (sp != 0) {
        sp--;
        long node_id = stk[3 * sp], left = stk[3 * sp + 1], right = stk[3 * sp + 2];
        bbox3 b = nb[node_id - 1];
        for (long i = left; i <= right; i++) b = merge_bb(b, bboxes[prims[i]]);
        nb[node_id - 1] = b;
        jt_bvh_node* nd = &nodes[node_id - 1];
        if (right - left + 1 > 4) { /* BVH_MAX_PRIMS (src/bvh.jl:32) */
            long mid;
            int axis;
            if (hq) split_sah(prims, bboxes, centers, left, right, &mid, &axis);
            else split_middle(prims, centers, left, right, &mid, &axis);
            long start = nnodes + 1;
            nd->start = (int32_t)(start - 1);
            nd->num = 2;
            nd->axis = (int8_t)(axis - 1);
            nd->internal = 1;
            nodes[nnodes].axis = 0; nb[nnodes] = bbox_empty(); nnodes++;
            nodes[nnodes].axis = 0; nb[nnodes] = bbox_empty(); nnodes++;
            stk[3 * sp] = start; stk[3 * sp + 1] = left; stk[3 * sp + 2] = mid; sp++;
            stk[3 * sp] = start + 1; stk[3 * sp + 1] = mid + 1; stk[3 * sp + 2] = right; sp++;
        } else {
            nd->start = (int32_t)(left - 1);
            nd->num = (int16_t)(right - left + 1);
            nd->internal = 0;
        }
    }
    for (long k = 0; k < nnodes; k++) {
        nodes[k].bmin[0] = nb[k].min.x; nodes[k].bmin[1] = nb[k].min.y; nodes[k].bmin[2] = nb[k].min.z;
        nodes[k].bmax[0] = nb[k].max.x; nodes[k].bmax[1] = nb[k].max.y; nodes[k].bmax[2] = nb[k].max.z;
    }
    out->nnodes = (int32_t)nnodes;
    out->nodes = nodes;
    out->nprimitives = (int32_t)n;
    out->primitives = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    for (long i = 1; i <= n; i++) out->primitives[i - 1] = (int32_t)(prims[i] - 1);
    free(prims);
    free(centers);
    free(stk);
    free(nb);
    return JT_OK;
}

int or_build_scene_bvh(const jt_scene* scene, int32_t high_quality, jt_scene_bvh* out) {
    memset(out, 0, sizeof(*out));
    out->nshapes = scene->nshapes;
    out->blas = (jt_bvh_tree*)calloc((size_t)(scene->nshapes > 0 ? scene->nshapes : 1), sizeof(jt_bvh_tree));
    for (int s = 0; s < scene->nshapes; s++) { /* make_shape_bvh (src/bvh.jl:90-136) */
        const jt_shape* sh = &scene->shapes[s];
        long n = 0;
        bbox3* bb = NULL;
        if (sh->ntriangles > 0) {
            n = sh->ntriangles;
            bb = (bbox3*)malloc(sizeof(bbox3) * (size_t)(n + 1));
            for (long i = 0; i < n; i++) {
                const int32_t* t = &sh->triangles[3 * i];
                bbox3 b; /* triangle_bounds: min.(p1, p2, p3) (src/geometry.jl:64) */
                b.min =V3(jl_min(jl_min(pos3(sh, t[0]).x, pos3(sh, t[1]).x), pos3(sh, t[2]).x),
                           jl_min(jl_min(pos3(sh, t[0]).y, pos3(sh, t[1]).y), pos3(sh, t[2]).y),
                           jl_min(jl_min(pos3(sh, t[0]).z, pos3(sh, t[1]).z), pos3(sh, t[2]).z));
                b.max = V3(jl_max(jl_max(pos3(sh, t[0]).x, pos3(sh, t[1]).x), pos3(sh, t[2]).x),
                           jl_max(jl_max(pos3(sh, t[0]).y, pos3(sh, t[1]).y), pos3(sh, t[2]).y),
                           jl_max(jl_max(pos3(sh, t[0]).z, pos3(sh, t[1]).z), pos3(sh, t[2]).z));
                bb[i + 1] = b;
            }
        } else if (sh->nquads > 0) {
            n = sh->nquads;
            bb = (bbox3*)malloc(sizeof(bbox3) * (size_t)(n + 1));
            for (long i = 0; i < n; i++) {
                const int32_t* q = &sh->quads[4 * i];
                v3 a = pos3(sh, q[0]), b2 = pos3(sh, q[1]), c = pos3(sh, q[2]), d = pos3(sh, q[3]);
                bbox3 b;
                b.min = V3(jl_min(jl_min(jl_min(a.x, b2.x), c.x), d.x), jl_min(jl_min(jl_min(a.y, b2.y), c.y), d.y),
                           jl_min(jl_min(jl_min(a.z, b2.z), c.z), d.z));
                b.max = V3(jl_max(jl_max(jl_max(a.x, b2.x), c.x), d.x), jl_max(jl_max(jl_max(a.y, b2.y), c.y), d.y),
                           jl_max(jl_max(jl_max(a.z, b2.z), c.z), d.z));
                bb[i + 1] = b;
            }
        } else {
            or_free_scene_bvh(out);
            return JT_ERR_UNSUPPORTED; /* points/lines/empty shapes */
        }
        int st = make_bvh(bb, n, high_quality, &out->blas[s]);
        free(bb);
        if (st != JT_OK) { or_free_scene_bvh(out); return st; }
    }
    long ni = scene->ninstances;
    bbox3* ib = (bbox3*)malloc(sizeof(bbox3) * (size_t)(ni + 1));
    for (long i = 0; i < ni; i++) { /* src/bvh.jl:77-85, transform_bbox (src/geometry.jl:70-86) */
        const jt_instance* inst = &scene->instances[i];
        const jt_bvh_tree* t = &out->blas[inst->shape];
        if (t->nnodes == 0) { ib[i + 1] = bbox_empty(); continue; }
        const jt_bvh_node* r = &t->nodes[0];
        fr3 f = frame_from(inst->frame);
        v3 corners[8] = {V3(r->bmin[0], r->bmin[1], r->bmin[2]), V3(r->bmin[0], r->bmin[1], r->bmax[2]),
                         V3(r->bmin[0], r->bmax[1], r->bmin[2]), V3(r->bmin[0], r->bmax[1], r->bmax[2]),
                         V3(r->bmax[0], r->bmin[1], r->bmin[2]), V3(r->bmax[0], r->bmin[1], r->bmax[2]),
                         V3(r->bmax[0], r->bmax[1], r->bmin[2]), V3(r->bmax[0], r->bmax[1], r->bmax[2])};
        bbox3 x = bbox_empty();
        for (int k = 0; k < 8; k++) x = merge_pt(x, transform_point(&f, corners[k]));
        ib[i + 1] = x;
    }
    int st = make_bvh(ib, ni, high_quality, &out->tlas);
    free(ib);
    if (st != JT_OK) { or_free_scene_bvh(out); return st; }
    return JT_OK;
}

void or_free_scene_bvh(jt_scene_bvh* bvh) {
    if (!bvh) return;
    free(bvh->tlas.nodes);
    free(bvh->tlas.primitives);
    if (bvh->blas) {
        for (int s = 0; s < bvh->nshapes; s++) {
            free(bvh->blas[s].nodes);
            free(bvh->blas[s].primitives);
        }
    }
    free(bvh->blas);
    memset(bvh, 0, sizeof(*bvh));
}

/* =========================================================== make_trace_lights (src/trace.jl:117-187) */
int or_make_lights(const jt_scene* scene, jt_lights* out) {
    memset(out, 0, sizeof(*out));
    int cap = scene->ninstances + scene->nenvironments + 1;
    out->lights = (jt_light*)calloc((size_t)cap, sizeof(jt_light));
    for (int h = 0; h < scene->ninstances; h++) {
        const jt_instance* inst = &scene->instances[h];
        const jt_material* m = &scene->materials[inst->material];
        if (m->emission[0] == 0 && m->emission[1] == 0 && m->emission[2] == 0) continue;
        const jt_shape* sh = &scene->shapes[inst->shape];
        if (sh->ntriangles == 0 && sh->nquads == 0) continue;
        jt_light* l = &out->lights[out->nlights++];
        l->instance = h;
        l->environment = -1;
        if (sh->nquads != 0) {
            l->ncdf = sh->nquads;
            l->cdf = (float*)malloc(sizeof(float) * (size_t)l->ncdf);
            for (int i = 0; i < sh->nquads; i++) {
                const int32_t* q = &sh->quads[4 * i];
                l->cdf[i] = quad_area(pos3(sh, q[0]), pos3(sh, q[1]), pos3(sh, q[2]), pos3(sh, q[3]));
                if (i != 0) l->cdf[i] += l->cdf[i - 1];
            }
        } else {
            l->ncdf = sh->ntriangles;
            l->cdf = (float*)malloc(sizeof(float) * (size_t)l->ncdf);
            for (int i = 0; i < sh->ntriangles; i++) {
                const int32_t* t = &sh->triangles[3 * i];
                l->cdf[i] = triangle_area(pos3(sh, t[0]), pos3(sh, t[1]), pos3(sh, t[2]));
                if (i != 0) l->cdf[i] += l->cdf[i - 1];
            }
        }
    }
    for (int h = 0; h < scene->nenvironments; h++) {
        const jt_environment* env = &scene->environments[h];
        if (env->emission[0] == 0 && env->emission[1] == 0 && env->emission[2] == 0) continue;
        if (env->emission_tex < 0) { or_free_lights(out); return JT_ERR_UNSUPPORTED; } /* UndefVarError */
        const jt_texture* tex = &scene->textures[env->emission_tex];
        jt_light* l = &out->lights[out->nlights++];
        l->instance = -1;
        l->environment = h;
        l->ncdf = tex->width * tex->height;
        l->cdf = (float*)malloc(sizeof(float) * (size_t)l->ncdf);
        for (long idx = 0; idx < l->ncdf; idx++) {
            long i = idx % tex->width, j = idx / tex->width;
            float th = ((float)j + 0.5f) * pif / (float)tex->height;
            v4 value = lookup_texture(tex, i, j, 0);
            float mv = jl_max(jl_max(jl_max(value.x, value.y), value.z), value.w);
            l->cdf[idx] = mv * jl_sin(th);
            if (idx != 0) l->cdf[idx] += l->cdf[idx - 1];
        }
    }
    return JT_OK;
}
void or_free_lights(jt_lights* lights) {
    if (!lights) return;
    if (lights->lights)
        for (int i = 0; i < lights->nlights; i++) free(lights->lights[i].cdf);
    free(lights->lights);
    memset(lights, 0, sizeof(*lights));
}

/* ============================================================== KAT entry points */
/* Property check of the wide records (JT_TRAVERSAL_WIDE) of every tree of a scene BVH, for the
 * tests: out[0] records, out[1] children whose dequantised box does NOT contain the exact box
 * (must be 0: the quantisation is conservative), out[2] leaves reached (must equal the binary
 * trees' leaves), out[3] the mean dequantised/exact volume ratio x 1000 over children with a
 * non-degenerate box (how loose the bytes make the boxes). */
static void w_check_tree(const jt_bvh_tree* b, const wtree_t* t, int64_t* out, double* vol, int64_t* nvol) {
    for (int r = 0; r < t->n; r++) {
        const wrec_t* w = &t->r[r];
        out[0]++;
        for (int k = 0; k < 4; k++) {
            if (w->child[k] < 0) continue;
            const jt_bvh_node* c = &b->nodes[w->child[k]];
            double ve = 1, vq = 1;
            for (int ax = 0; ax < 3; ax++) {
                float lo = w->o[ax] + (float)w->lo[ax][k] * w->s[ax];
                float hi = w->o[ax] + (float)w->hi[ax][k] * w->s[ax];
                if (!(lo <= c->bmin[ax] && hi >= c->bmax[ax])) out[1]++;
                ve *= (double)c->bmax[ax] - (double)c->bmin[ax];
                vq *= (double)hi - (double)lo;
            }
            if (!c->internal) out[2]++;
            if (ve > 0) { *vol += vq / ve; (*nvol)++; }
        }
    }
}
int or_wide_check(const jt_bvh_tree* tlas, const jt_bvh_tree* blas, int32_t nblas, int64_t* out) {
    double vol = 0;
    int64_t nvol = 0;
    out[0] = out[1] = out[2] = out[3] = 0;
    for (int i = -1; i < nblas; i++) {
        const jt_bvh_tree* b = i < 0 ? tlas : &blas[i];
        if (b->nnodes == 0) continue;
        wtree_t t = {0, 0, NULL};
        if (w_build(b, 0, &t) < 0) { free(t.r); return JT_ERR_UNSUPPORTED; }
        w_check_tree(b, &t, out, &vol, &nvol);
        free(t.r);
    }
    out[3] = nvol ? (int64_t)(1000.0 * vol / (double)nvol) : 0;
    return JT_OK;
}

int or_intersect_triangle(const float* o, const float* d, float tmin, float tmax, const float* p1, const float* p2,
                          const float* p3, float* out_uvt) {
    ray3 r = {V3(o[0], o[1], o[2]), V3(d[0], d[1], d[2]), tmin, tmax};
    prim_isec p = intersect_triangle(&r, V3(p1[0], p1[1], p1[2]), V3(p2[0], p2[1], p2[2]), V3(p3[0], p3[1], p3[2]));
    out_uvt[0] = p.uv.x;
    out_uvt[1] = p.uv.y;
    out_uvt[2] = p.distance;
    return p.hit;
}
int or_intersect_bbox(const float* o, const float* d, float tmin, float tmax, const float* bmin, const float* bmax) {
    ray3 r = {V3(o[0], o[1], o[2]), V3(d[0], d[1], d[2]), tmin, tmax};
    v3 dinv = V3(1 / d[0], 1 / d[1], 1 / d[2]);
    return intersect_bbox(&r, dinv, bmin, bmax);
}
float or_fresnel_dielectric(float eta, const float* normal, const float* outgoing) {
    return fresnel_dielectric(eta, V3(normal[0], normal[1], normal[2]), V3(outgoing[0], outgoing[1], outgoing[2]));
}
void or_rng_first(uint64_t seed, int32_t pixel, int32_t sample, int32_t n, float* out) {
    rng_t r = rng_init(seed, pixel, sample);
    for (int i = 0; i < n; i++) out[i] = rand1f(&r);
}
void or_inverse_frame(const float* frame, int32_t non_rigid, float* out) {
    fr3 f = frame_from(frame);
    fr3 r = inverse_frame(&f, non_rigid);
    float v[12] = {r.x.x, r.x.y, r.x.z, r.y.x, r.y.y, r.y.z, r.z.x, r.z.y, r.z.z, r.o.x, r.o.y, r.o.z};
    memcpy(out, v, sizeof(v));
}
void or_srgb_to_rgb(const uint8_t* bytes, int32_t n, float* out) {
    for (int i = 0; i < n; i++) out[i] = srgb_to_rgb1(bytes[i] / 255.0f);
}
