// jt_device.h — device-side data layout and per-lane math of the MI355X path tracer.
//
// Everything here runs per lane inside the trace megakernel (jt_trace.hip). Each function
// cites the reference (Princic-1837592/julia-raytracer) source it computes. Float contract
// (DESIGN.md §Numerics): compiled with -ffp-contract=off (no FMA contraction, Julia's
// evaluation order), Julia's NaN-propagating min/max, and — in the parity build
// (JT_EXACT_MATH=1, the default) — transcendentals evaluated in double and rounded once,
// which is how Julia's Float32 kernels compute them.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// automatic stream count (jt_trace.hip stream_log2): at least JT_STREAMS_MIN streams —
// JT_STREAMS_WIDE for a batch of at least two samples per such stream — and JT_STREAM_ITEMS
// (pixel, stream) items, at most JT_STREAM_ITEMS_MAX items
#define JT_STREAMS_MIN 16
#define JT_STREAMS_WIDE 32
#define JT_STREAM_ITEMS (1LL << 22)
#define JT_STREAM_ITEMS_MAX (1LL << 27)
#ifndef JT_AUTO_WIDE_MIN_STACK
#define JT_AUTO_WIDE_MIN_STACK 32  // JT_TRAVERSAL_AUTO: wide records for HBM-mode scenes deeper than this
#endif
// jt_trace_range defers its range until this many samples are queued (jt_ctx::pend0)
#define JT_DEFER_SAMPLES 64
#ifndef JT_MAX_STREAMS
#define JT_MAX_STREAMS 64  // sample streams per pixel (a power of two, jt_ctx::streams)
#endif
#ifndef JT_EXACT_MATH
#define JT_EXACT_MATH 1
#endif

namespace jtd {

// ------------------------------------------------------------------------------ layout in HBM
// BVH node, 32 B = two 16-B loads: a = (bmin.x, bmax.x, bmin.y, bmax.y), b = (bmin.z, bmax.z,
// start bits, meta bits), each axis's slab planes side by side. meta = num | axis << 16 |
// internal << 24. TLAS nodes come first (breadth-first), then every BLAS; `start` is a global
// node index (internal), a triangle-pair / quad record slot (BLAS leaf) or, for a TLAS leaf, its
// first instance: the device numbers instances in TLAS leaf order (bvh.primitives[i] of the
// reference becomes instance i), so a leaf's instances are start .. start+num-1.
struct alignas(16) DNode {
    float4 a, b;
};
// Wide (4-ary) node record, 64 B = four 16-B loads: the traversal jt_params.traversal =
// JT_TRAVERSAL_WIDE. A record stands for an internal binary node N of the
// reference's tree (or a leaf root) and holds N's grandchildren: N's two children, each internal
// child replaced by its own two children, so one visit tests up to four boxes and a DFS visits the
// reference's leaves in the binary order. The boxes are conservative 8-bit quantisations relative
// to N's box (dequantised lo = origin + q * scale in float, never above the exact bmin; hi never
// below bmax), tested with the reference's intersect_bbox:
//   r0: origin.xyz = N's bmin, meta bits = ex | ey << 8 | ez << 16 | (a0 | a1 << 2 | a2 << 4) << 24
//       (scale of an axis = the float with biased exponent e, 2^(e - 127); a0 = N's split axis,
//       a1 / a2 the split axes of N's children L / R, 0 for a leaf child)
//   r1: bytes lo.x[4] hi.x[4] lo.y[4] hi.y[4] of slots 0..3; r2: lo.z[4] hi.z[4], 0, 0
//   r3: child words of slots [LL, LR, RL, RR] (a leaf child L / R takes slot 0 / 2 alone)
// child word: W_EMPTY; bit 31 clear: a record index; bit 31 set: a leaf, bit 30 set for a TLAS
// leaf (instances start .. start + num - 1), bits 28-29 num - 1, bits 0-27 start (first instance,
// triangle-pair record or quad record)
struct alignas(16) DWide {
    float4 r0;
    uint4 r1, r2;
    uint4 r3;
};
enum : unsigned { W_EMPTY = 0xffffffffu, W_LEAF = 0x80000000u, W_INST = 0x40000000u, W_START = 0x0fffffffu };
// Traversal record of an instance, 64 B: inverse(frame, true) as 12 floats + ids.
struct alignas(16) DInstTrav {
    float4 i0, i1, i2;  // inv x.xyz y.x | y.yz z.xy | z.z o.xyz
    int shape, blas_root, kind, prim_base;
};
// Shading record of an instance, 64 B: frame (12 floats) + material / shape ids.
struct alignas(16) DInstShade {
    float4 f0, f1, f2;
    int material, shape, mat_type;
    int rot_identity;  // frame x, y, z are exactly the unit axes: element normals from enrm_id
};
enum { KIND_TRI = 0, KIND_QUAD = 1 };
// Scene feature bits of a kernel specialisation (chosen per scene by jt_create): a kernel built
// without a bit assumes the scene has none of it, so the branches it guards are compiled out.
// FT_ALL is the general kernel; FT_NONE serves scenes of matte triangles without textures,
// vertex attributes, environments or opacity (cornellbox); jt_create picks the smallest compiled
// mask that covers the scene (jt_trace.hip, launch_s). Results are bit-identical.
enum : int {
    FT_TEX = 1,    // material textures (incl. normal maps)
    FT_ATTR = 2,   // shape normals / texcoords / colors
    FT_QUAD = 4,   // quad shapes
    FT_MAT = 8,    // materials other than matte
    FT_ENV = 16,   // environments (escaped rays, environment lights)
    FT_OPAC = 32,  // opacity < 1 possible (material opacity, color-texture or vertex-color alpha)
    FT_VOL = 64,   // refractive / subsurface / volumetric materials (the volume stack)
    FT_XFORM = 128,  // instances whose inverse frame is not exactly the identity
    FT_NONE = 0,
    FT_ALL = 255,
    // kernel build flag, not a scene feature: the scene's light chains run inline
    // (DScene::light_inline; jt_kernels.h light_chain), so the kernel has no light-hit steps
    FT_LINL = 8192,
    // kernel build flag: the scene has no instance light (sample_lights_pdf never queries a BVH)
    FT_NOIL = 16384
};
// a kernel mask of no scene feature (the FT_NONE kernels, with or without the FT_LINL build flag)
__host__ __device__ constexpr bool ft_none(int F) { return (F & ~(FT_LINL | FT_NOIL)) == FT_NONE; }
struct alignas(16) DShape {
    int kind, blas_root, prim_base, idx_base;
    int pos_base, nrm_base, tc_base, col_base;  // -1 = absent
};
struct alignas(16) DMaterial {
    int type, emission_tex, color_tex, roughness_tex;
    int scattering_tex, normal_tex, pad0, pad1;
    float emission[3], roughness;
    float color[3], metallic;
    float scattering[3], ior;
    float scanisotropy, trdepth, opacity, pad2;
};
struct alignas(16) DTexture {
    int width, height, linear, is_float;
    long long offset;  // texel index into texb (uchar4) or texf (float4)
    long long pad;
};
struct alignas(16) DEnv {
    float frame[12];
    float inv[12];  // inverse(frame) rigid (src/scene.jl:906)
    float emission[3];
    int tex;
};
// One element of an instance light, as light_hit reads it (5 float4): its object-space vertex
// positions p1 p2 p3 (p4 for a quad in row 4), the element normal light_hit transforms (enrm, or
// enrm_id already final when the instance frame has no rotation), the light's area (last of its
// CDF), the rot_identity flag and the shape kind. The same floats as the arrays they come from:
// light_hit's results are unchanged, from 4-5 loads instead of 10.
//   row 0: p1.xyz p2.x | row 1: p2.yz p3.xy | row 2: p3.z n.xyz | row 3: area rot kind 0 | row 4: p4.xyz 0
struct alignas(16) DLight {
    int instance, environment, cdf_offset, ncdf;
    // guide table of a long CDF (env lights; nguide = 0: plain binary search): thresholds
    // guide_t[k] (float) and guide_a[k] = first 0-based index i with cdf[i] > guide_t[k]
    int guide_offset, nguide;
    float guide_scale;  // nguide / last(cdf): first guess of the bucket of a limit
    // JT_ENV_ALIAS=1 (statistical variant, not the default): offset of an environment light's
    // Vose alias table in DScene::alias (ncdf entries), -1 = none
    int alias_offset;
};

struct DScene {
    const DNode* nodes;      // TLAS nodes, then every BLAS (global node indices)
    const DWide* wnodes;     // the wide traversal's records: TLAS records, then every BLAS's
    int tlas_wnodes;         // TLAS records (a record index below it is a TLAS record)
    const float4* prims;  // triangle pair: 5 float4 (p1, p2-p1, p3-p1 of two triangles interleaved,
                          // then both element ids); quad: 4 float4 (p1|elem, p2, p3, p4|p3==p4)
    const DInstTrav* inst_trav;
    const int4* inst_blas;  // per instance: blas_root, identity-transform flag, kind, shape
    const DInstShade* inst_shade;
    const DShape* shapes;
    const float4* pos;
    const float4* nrm;
    const float2* tc;
    const float4* col;
    const int4* elems;  // triangle (a,b,c,0) / quad (a,b,c,d), global vertex ids
    // per element, precomputed on the host with the device's float operations:
    // triangle_normal / quad_normal in object space, and transform_normal of it by an
    // identity-rotation frame (eval_element_normal of an instance whose frame has no rotation)
    const float4* enrm;
    const float4* enrm_id;
    const DMaterial* materials;
    const DTexture* textures;
    const uchar4* texb;
    const float4* texf;
    const DEnv* envs;
    const DLight* lights;
    // light-hit records (light_hit, src/trace.jl:1024-1044): per light (instance, first record,
    // 0, 0), and per element of an instance light's shape one 80-B record of what light_hit
    // reads, gathered on the host (DLightElem)
    const int4* light_hit;
    const float4* light_elems;
    const float* cdf;
    const float* guide_t;   // DLight guide tables (thresholds / first indices)
    const int* guide_a;
    const float2* alias;    // DLight alias tables: (keep probability, alias index bits) per texel
    const float* srgb_lut;  // srgb_to_rgb(byte_to_float(b)), 256 entries (src/color.jl:12-23)
    const float* byte_lut;  // byte_to_float(b)
    int tlas_nnodes, nenvs, nlights;
    int order_flip;  // jt_params.traversal: 0 the reference's child order, 7 the near child first
                     // (near and wide)
    float light_pick_pdf;  // sample_uniform_pdf(nlights) = Float32(1 / nlights) (src/sampling.jl:31)
    int light_inline;  // every instance light's shape BVH is one leaf: light chains run inline (jtk::light_chain)
    // Small-scene mode: every array above that the traversal and shading read per step, packed
    // in one 16-B aligned blob the workgroup copies into LDS at kernel start (offsets in 16-B
    // units; -1 = not in the blob). Texels, environments and LUTs stay in HBM.
    const uint4* blob;
    int blob_n16;
    // traversal-stack overflow (scenes deeper than the LDS ring): ovf_stride entries per pixel
    int* ovf;
    int ovf_stride;
    int ring;  // entries of the LDS ring in use (a power of two <= the kernel's RING)
    int stack_need;  // stack bound of the scene: LDS-mode kernels without overflow allocate this many
    int o_wnodes;
    int o_nodes, o_prims, o_inst_trav, o_inst_blas, o_inst_shade, o_shapes;
    int o_pos, o_nrm, o_tc, o_col, o_elems, o_materials, o_lights, o_cdf, o_enrm, o_enrm_id;
    int o_light_hit, o_light_elems;
};

struct DCamera {
    float frame[12];
    int orthographic;
    float lens, film, aspect, focus, aperture;
    float film_x, film_y;  // the film vector of eval_camera (src/scene.jl:377-378), host-computed
    int pinhole;           // aperture is +0: only the signs of sample_disk matter
};

struct DParams {
    DCamera cam;
    int width, height;
    int bounces, sampler;
    float clamp;
    int envhidden, tentfilter, nocaustics;
    int first;  // running-mean origin: local sample t = s - first
    // sample streams (DESIGN.md §2 "Sample streams"): local sample t belongs to stream
    // t & (2^lk - 1) and is the (t >> lk)-th sample of that stream's own running mean, weight
    // 1/((t >> lk) + 1); the launch ends by combining the streams' means (jt_trace.hip combine)
    int lk;
    int wait_lanes;
    int light_lanes;  // path sampler: run a light-hit step inside the traversal phase once this
                      // many lanes wait on a sample_lights_pdf query result (65: never)
    // the 8x8 tiles this launch covers: t = k * tile_stride + tile_offset (a multi-device context
    // split by pixel tiles, jt_create_multi; 1 / 0 otherwise: every tile)
    int tile_stride, tile_offset;
    unsigned long long seed;
};

// ------------------------------------------------------------------------------ math (src/math.jl)
static constexpr float pif = 3.14159265358979323846f;  // Float32(pi)
static constexpr float ray_eps = 0.0001f;               // src/geometry.jl:34
static constexpr float min_roughness = 0.03f * 0.03f;   // src/scene.jl:46

struct v2 {
    float x, y;
};
struct v3 {
    float x, y, z;
};
struct v4 {
    float x, y, z, w;
};

__device__ __forceinline__ v2 V2(float x, float y) { return v2{x, y}; }
__device__ __forceinline__ v3 V3(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v4 V4(float x, float y, float z, float w) { return v4{x, y, z, w}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 operator*(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 operator*(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ v3 operator/(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ v3 operator-(v3 a) { return V3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ v4 operator+(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ v4 operator*(v4 a, float s) { return V4(a.x * s, a.y * s, a.z * s, a.w * s); }
__device__ __forceinline__ bool is_zero(v3 a) { return a.x == 0 && a.y == 0 && a.z == 0; }
__device__ __forceinline__ bool all_finite(v3 a) {
    return __builtin_isfinite(a.x) && __builtin_isfinite(a.y) && __builtin_isfinite(a.z);
}
__device__ __forceinline__ v3 xyz(float4 a) { return V3(a.x, a.y, a.z); }
__device__ __forceinline__ v3 xyz(v4 a) { return V3(a.x, a.y, a.z); }

// dot = sum(a .* b), left fold (src/math.jl:69)
__device__ __forceinline__ float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ v3 cross(v3 a, v3 b) {  // src/math.jl:112
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ v3 normalize(v3 a) {  // src/math.jl:71-78
    float l = __builtin_sqrtf(dot(a, a));
    return l != 0 ? a / l : a;
}
__device__ __forceinline__ float length(v3 a) { return __builtin_sqrtf(dot(a, a)); }

// Julia min/max for floats (base/math.jl): NaN-propagating, -0 < +0 — IEEE 754-2019
// minimum/maximum, which gfx950 has as v_minimum3_f32 / v_maximum3_f32 (JT_NAN_PROP, one
// instruction; the compare-and-select form otherwise). A NaN result may carry another payload than
// Julia's (x's or y's): no decision and no stored value depends on a NaN's payload.
#ifndef JT_NAN_PROP
#define JT_NAN_PROP 1
#endif
__device__ __forceinline__ float jl_min3(float a, float b, float c) {
    float r;
    asm("v_minimum3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float jl_max3(float a, float b, float c) {
    float r;
    asm("v_maximum3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float jl_min(float x, float y) {
    if (JT_NAN_PROP) return jl_min3(x, y, y);
    bool c = (y < x) || (__builtin_signbit(y) && !__builtin_signbit(x));
    return c ? (__builtin_isnan(x) ? x : y) : (__builtin_isnan(y) ? y : x);
}
__device__ __forceinline__ float jl_max(float x, float y) {
    if (JT_NAN_PROP) return jl_max3(x, y, y);
    bool c = (y > x) || (!__builtin_signbit(y) && __builtin_signbit(x));
    return c ? (__builtin_isnan(x) ? x : y) : (__builtin_isnan(y) ? y : x);
}
__device__ __forceinline__ float jl_clamp(float x, float lo, float hi) { return x > hi ? hi : (x < lo ? lo : x); }
// 1.0f / x, correctly rounded like the IEEE division it replaces: v_rcp_f32 plus one FMA Newton
// step equals it for every x with a normal exponent below 2^126 (so the reciprocal is normal
// too) — verified over all 2^32 inputs by scripts/exhaustive/rcp_check.hip on gfx950. Zeros,
// denormals, |x| >= 2^126, inf and NaN take the division.
__device__ __forceinline__ float jl_rcp(float x) {
    const unsigned e = (__float_as_uint(x) >> 23) & 0xffu;
    if (__builtin_expect(e - 1u < 252u, 1)) {
        const float r = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    }
    return 1.0f / x;
}
__device__ __forceinline__ int jl_clampi(int x, int lo, int hi) { return x > hi ? hi : (x < lo ? lo : x); }
__device__ __forceinline__ float max3(v3 a) { return JT_NAN_PROP ? jl_max3(a.x, a.y, a.z) : jl_max(jl_max(a.x, a.y), a.z); }

#if JT_EXACT_MATH
// Double-evaluated, once-rounded transcendentals (the float contract). The hot-path arguments
// of sin/cos (2*pi*u, atan(...), v*pi, u*2*pi) lie in [0, 2*pi]; for |x| < 2^19 a Cody-Waite
// reduction by pi/2 with a 33-bit leading constant is exact in double and the fdlibm kernels
// give < 1 ulp in double, so rounding to float reproduces the correctly rounded float except
// within ~2^-52 of a rounding midpoint. Larger arguments fall back to ocml's double sincos.
__device__ __forceinline__ void dsincos_small(double x, double& s, double& c) {
    const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11;
    const double n = __builtin_rint(x * invpio2);
    const double r = (x - n * pio2_1) - n * pio2_1t;
    const double z = r * r;
    // __kernel_sin / __kernel_cos (fdlibm k_sin.c / k_cos.c), tail y = 0
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double sr = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double ks = r + (z * r) * (S1 + z * sr);
    const double cr = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double kc = w + (((1.0 - w) - hz) + z * cr);
    const int q = (int)n & 3;
    s = q == 0 ? ks : (q == 1 ? kc : (q == 2 ? -ks : -kc));
    c = q == 0 ? kc : (q == 1 ? -ks : (q == 2 ? -kc : ks));
}
__device__ __noinline__ void dsincos_large(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ void jl_sincos(float x, float* s, float* c) {
    double sd, cd;
    if (__builtin_fabsf(x) < 524288.0f) {
        dsincos_small((double)x, sd, cd);
    } else {
        dsincos_large((double)x, &sd, &cd);
    }
    *s = (float)sd;
    *c = (float)cd;
}
__device__ __forceinline__ float jl_sin(float x) {
    float s, c;
    jl_sincos(x, &s, &c);
    return s;
}
__device__ __forceinline__ float jl_cos(float x) {
    float s, c;
    jl_sincos(x, &s, &c);
    return c;
}
// atan in double (fdlibm s_atan.c), used by sample_microfacet on every rough specular sample
__device__ __forceinline__ float jl_atan(float xf) {
    const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                              1.57079632679489655800e+00};
    const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                              6.12323399573676603587e-17};
    const double a0 = 3.33333333333329318027e-01, a1 = -1.99999999998764832476e-01, a2 = 1.42857142725034663711e-01,
                 a3 = -1.11111104054623557880e-01, a4 = 9.09088713343650656196e-02, a5 = -7.69187620504482999495e-02,
                 a6 = 6.66107313738753120669e-02, a7 = -5.83357013379057348645e-02, a8 = 4.97687799461593236017e-02,
                 a9 = -3.65315727442169155270e-02, a10 = 1.62858201153657823623e-02;
    if (__builtin_isnan(xf)) return xf;
    const double x0 = (double)xf;
    double x = __builtin_fabs(x0);
    int id;
    if (x < 0.4375) {
        if (x < 1.0e-29) return xf;
        id = -1;
    } else if (x < 1.1875) {
        if (x < 0.6875) {
            id = 0;
            x = (2.0 * x - 1.0) / (2.0 + x);
        } else {
            id = 1;
            x = (x - 1.0) / (x + 1.0);
        }
    } else if (x < 2.4375) {
        id = 2;
        x = (x - 1.5) / (1.0 + 1.5 * x);
    } else if (x < 1.0e17) {
        id = 3;
        x = -1.0 / x;
    } else {
        return (float)__builtin_copysign(atanhi[3] + atanlo[3], x0);
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
    const double s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
    double r;
    if (id < 0) r = x - x * (s1 + s2);
    else r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (float)__builtin_copysign(r, x0);
}
// rare-path transcendentals (environment, volumes): ocml double, kept out of line
__device__ __noinline__ float jl_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
__device__ __noinline__ float jl_acos(float x) { return (float)acos((double)x); }
__device__ __noinline__ float jl_log(float x) { return (float)log((double)x); }
__device__ __noinline__ float jl_exp(float x) { return (float)exp((double)x); }
#else
__device__ __forceinline__ float jl_sin(float x) { return sinf(x); }
__device__ __forceinline__ float jl_cos(float x) { return cosf(x); }
__device__ __forceinline__ void jl_sincos(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ float jl_atan(float x) { return atanf(x); }
__device__ __forceinline__ float jl_atan2(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ float jl_acos(float x) { return acosf(x); }
__device__ __forceinline__ float jl_log(float x) { return logf(x); }
__device__ __forceinline__ float jl_exp(float x) { return expf(x); }
#endif

// Frame3f columns x, y, z, o packed in 12 floats
struct fr3 {
    v3 x, y, z, o;
};
__device__ __forceinline__ fr3 frame_from(const float* a) {
    return fr3{V3(a[0], a[1], a[2]), V3(a[3], a[4], a[5]), V3(a[6], a[7], a[8]), V3(a[9], a[10], a[11])};
}
__device__ __forceinline__ fr3 frame_from(float4 a, float4 b, float4 c) {
    return fr3{V3(a.x, a.y, a.z), V3(a.w, b.x, b.y), V3(b.z, b.w, c.x), V3(c.y, c.z, c.w)};
}
// transform_point / transform_vector / transform_direction / transform_normal (src/math.jl:80-129)
__device__ __forceinline__ v3 transform_point(const fr3& f, v3 p) { return ((f.x * p.x + f.y * p.y) + f.z * p.z) + f.o; }
__device__ __forceinline__ v3 transform_vector(const fr3& f, v3 b) { return (f.x * b.x + f.y * b.y) + f.z * b.z; }
__device__ __forceinline__ v3 transform_direction(const fr3& f, v3 b) { return normalize(transform_vector(f, b)); }
__device__ __forceinline__ v3 transform_normal(const fr3& f, v3 b) { return normalize(transform_vector(f, b)); }
// Mat3f (3 columns) * Vec3f (src/math.jl:105)
struct m3 {
    v3 c1, c2, c3;
};
__device__ __forceinline__ v3 mul(const m3& m, v3 f) { return (m.c1 * f.x + m.c2 * f.y) + m.c3 * f.z; }
// reflect / refract (src/math.jl:131-142)
__device__ __forceinline__ v3 reflect(v3 w, v3 n) { return -w + n * (2 * dot(n, w)); }
__device__ __forceinline__ v3 refract(v3 w, v3 n, float inv_eta) {
    float cosine = dot(n, w);
    float k = 1 + inv_eta * inv_eta * (cosine * cosine - 1);
    if (k < 0) return V3(0, 0, 0);
    return (-w) * inv_eta + n * (inv_eta * cosine - __builtin_sqrtf(k));
}

// ------------------------------------------------------------------------------ RNG (build)
// PCG32 stream keyed by (seed, pixel, global sample); rand1f = 24-bit float in [0,1) like
// Julia's rand(Float32). Stated in DESIGN.md §RNG and restated by oracle/jt_oracle.c.
struct Rng {
    unsigned long long state, inc;
};
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ Rng rng_init(unsigned long long seed, int pixel, int sample) {
    unsigned long long key = mix64(seed ^ mix64(((unsigned long long)(unsigned)pixel << 32) |
                                                 (unsigned long long)(unsigned)sample));
    Rng r;
    r.inc = (mix64(key ^ 0xda3e39cb94b95bdbULL) << 1) | 1ULL;
    r.state = (r.inc + key) * 6364136223846793005ULL + r.inc;
    return r;
}
__device__ __forceinline__ unsigned rng_next(Rng& r) {
    unsigned long long old = r.state;
    r.state = old * 6364136223846793005ULL + r.inc;
    unsigned xs = (unsigned)(((old >> 18) ^ old) >> 27);
    unsigned rot = (unsigned)(old >> 59);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}
__device__ __forceinline__ float rand1f(Rng& r) { return (float)(rng_next(r) >> 8) * 0x1.0p-24f; }
__device__ __forceinline__ v2 rand2f(Rng& r) {
    float a = rand1f(r);
    float b = rand1f(r);
    return V2(a, b);
}

// ------------------------------------------------------------------------------ sampling.jl
__device__ __forceinline__ v2 sample_disk(v2 ruv) {  // src/sampling.jl:12-16
    float r = __builtin_sqrtf(ruv.y);
    float phi = 2 * pif * ruv.x;
    float s, c;
    jl_sincos(phi, &s, &c);
    return V2(c * r, s * r);
}
// With aperture == +0, eval_camera reads sample_disk's result only through lens_uv * 0, i.e.
// through the signs of c * r and s * r (r >= +0): those of cos(phi) and sin(phi). The float phi
// is compared in double against the doubles nearest pi/2, pi, 3pi/2, 2pi; no float lies
// between any of them and the true value, and cos/sin of a float are never zero except
// sin(+0), so the signs are exactly those of the rounded jl_sincos results.
__device__ __forceinline__ v2 sample_disk_signs(v2 ruv) {
    const double phi = (double)(2 * pif * ruv.x);
    const bool cneg = phi > 1.5707963267948966 && phi < 4.7123889803846897;
    const bool sneg = phi > 3.1415926535897931 && phi < 6.2831853071795862;
    return V2(cneg ? -0.0f : 0.0f, sneg ? -0.0f : 0.0f);
}
__device__ __forceinline__ float sample_hemisphere_cos_pdf(v3 normal, v3 direction) {  // :24-27
    float cosw = dot(normal, direction);
    return cosw <= 0 ? 0 : cosw / pif;
}
__device__ __forceinline__ int sample_uniform(int size, float r) {  // :29, 1-based
    return jl_clampi((int)__builtin_truncf(r * (float)size) + 1, 1, size);
}
__device__ __forceinline__ float sample_uniform_pdf(int size) { return (float)(1.0 / (double)size); }  // :31
__device__ __forceinline__ int upper_bound(const float* cdf, int n, float limit) {  // :42-56, 1-based
    int idx = 0, l = 1, r = n;
    while (l <= r) {
        int m = (l + r) / 2;
        if (cdf[m - 1] > limit) {
            idx = m;
            r = m - 1;
        } else {
            l = m + 1;
        }
    }
    return idx;
}
__device__ __forceinline__ int sample_discrete(const float* cdf, int n, float r) {  // :33-37, 1-based
    float last = cdf[n - 1];
    r = jl_clamp(r * last, 0.0f, last - 0.00001f);
    return jl_clampi(upper_bound(cdf, n, r), 1, n);
}
// upper_bound through a guide table: the same first index (cdf is nondecreasing, so the answer
// for a limit in [t_k, t_k+1) lies in [a_k, a_k+1]); a few loads instead of log2(n) dependent ones
__device__ __forceinline__ int upper_bound_guided(const float* cdf, int n, float limit, const float* gt, const int* ga,
                                                  int K, float scale) {
    int k = (int)(limit * scale);
    k = k < 0 ? 0 : (k > K - 1 ? K - 1 : k);
    while (k > 0 && limit < gt[k]) k--;
    while (k < K - 1 && limit >= gt[k + 1]) k++;
    int lo = ga[k], hi = ga[k + 1];
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] > limit) hi = mid;
        else lo = mid + 1;
    }
    return lo >= n ? 0 : lo + 1;
}
__device__ __forceinline__ int sample_discrete_guided(const float* cdf, int n, float r, const float* gt, const int* ga,
                                                      int K, float scale) {
    float last = cdf[n - 1];
    r = jl_clamp(r * last, 0.0f, last - 0.00001f);
    return jl_clampi(upper_bound_guided(cdf, n, r, gt, ga, K, scale), 1, n);
}
__device__ __forceinline__ float sample_discrete_pdf(const float* cdf, int idx1) {  // :39-40
    return idx1 == 1 ? cdf[0] : cdf[idx1 - 1] - cdf[idx1 - 2];
}
__device__ __forceinline__ v2 sample_triangle(v2 ruv) {  // :58
    return V2(1 - __builtin_sqrtf(ruv.x), ruv.y * __builtin_sqrtf(ruv.x));
}

// ------------------------------------------------------------------------------ geometry.jl
// Raw VALU min/max. Only for operands known not to be NaN: the compiler's fminf/fmaxf
// canonicalize both inputs first (IEEE mode), which costs an extra VALU op per operand.
__device__ __forceinline__ float vmin(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmin3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// The slab test's final compare, `t1 *= 1.00000024; t0 <= t1` (src/geometry.jl:102-103): the
// Float32 t1 is promoted, so the product and the compare are Float64. (An exact float decision
// with a double fallback — checked exhaustively, scripts/exhaustive/slab_check.hip — measured
// slower on gfx950, whose wave64 FP64 multiply issues at the FP32 rate)
__device__ __forceinline__ bool slab_pass(float t0, float t1) { return (double)t0 <= (double)t1 * 1.00000024; }

// intersect_bbox (src/geometry.jl:96-105): Julia min/max; `t1 *= 1.00000024` is Float64.
// Any NaN slab value makes Julia's t0 or t1 NaN and culls the box; that case is tested
// separately, so the min/max chains below only ever see non-NaN values, where IEEE min/max
// agree with Julia's (signed zeros cannot change `t0 <= t1`) and the order of the chain does
// not matter.
// a = (bmin.x, bmax.x, bmin.y, bmax.y), b = (bmin.z, bmax.z, ..) (DNode). Scalar on purpose:
// packed-FP32 (v_pk_add/v_pk_mul_f32) forms of these products measured 1.5 % slower on gfx950
// (the broadcast ray operands then occupy register pairs).
// JT_NAN_PROP (jl_min above): with Julia's min/max as single NaN-propagating instructions a NaN
// slab value makes t0 or t1 NaN and the Float64 compare false, with no separate NaN test (three
// v_cmp_o and their mask combines per box): the same decision as the form below for every input.
// Measured against it (two runs each, interleaved, gpurun_out/r06nan2): cornellbox +1.5 %,
// bathroom1 +1.6 %, ecosys +1.0 %, features2 +1.3 %.
__device__ __forceinline__ bool intersect_bbox(v3 o, v3 dinv, float tmin, float tmax, const float4& a,
                                               const float4& b) {
    const float mx = (a.x - o.x) * dinv.x, Mx = (a.y - o.x) * dinv.x;
    const float my = (a.z - o.y) * dinv.y, My = (a.w - o.y) * dinv.y;
    const float mz = (b.x - o.z) * dinv.z, Mz = (b.y - o.z) * dinv.z;
    if (JT_NAN_PROP) {
        // t0 = max(min(mx, Mx), min(my, My), max(min(mz, Mz), tmin)), t1 likewise (the order of a
        // max chain does not change its value; a NaN anywhere makes it NaN)
        const float t0 = jl_max3(jl_min3(mx, Mx, Mx), jl_min3(my, My, My), jl_max3(jl_min3(mz, Mz, Mz), tmin, tmin));
        const float t1 = jl_min3(jl_max3(mx, Mx, Mx), jl_max3(my, My, My), jl_min3(jl_max3(mz, Mz, Mz), tmax, tmax));
        return slab_pass(t0, t1);
    }
    bool nan = __builtin_isnan(mx) | __builtin_isnan(my) | __builtin_isnan(mz) | __builtin_isnan(Mx) |
               __builtin_isnan(My) | __builtin_isnan(Mz);
    float t0 = vmax3(vmin(mx, Mx), vmin(my, My), vmax(vmin(mz, Mz), tmin));
    float t1 = vmin3(vmax(mx, Mx), vmax(my, My), vmin(vmax(mz, Mz), tmax));
    return !nan && slab_pass(t0, t1);
}

struct PrimHit {
    float u, v, t;
    bool hit;
};
// intersect_triangle (src/geometry.jl:206-236), branchless: every quantity is computed and the
// reference's early-out tests are combined into one predicate (the same comparisons, so NaN
// behaves as in the reference: a NaN u, v or t fails none of them). A miss is (0, 0, inf).
__device__ __forceinline__ PrimHit intersect_triangle_e(v3 o, v3 d, float tmin, float tmax, v3 p1, v3 edge1, v3 edge2) {
    v3 pvec = cross(d, edge2);
    float det = dot(edge1, pvec);
    float inv_det = jl_rcp(det);
    v3 tvec = o - p1;
    float u = dot(tvec, pvec) * inv_det;
    v3 qvec = cross(tvec, edge1);
    float v = dot(d, qvec) * inv_det;
    float t = dot(edge2, qvec) * inv_det;
    const bool miss = (det == 0) | (u < 0 || u > 1) | (v < 0 || u + v > 1) | (t < tmin || t > tmax);
    PrimHit r;
    r.u = miss ? 0.0f : u;
    r.v = miss ? 0.0f : v;
    r.t = miss ? __builtin_inff() : t;
    r.hit = !miss;
    return r;
}
// The triangle test without its `t > tmax` rejection (the only use of tmax): hit = every other
// test passed. tri_hit_before(p, tmax) completes it, so two consecutive primitives can be
// computed side by side and then accepted in order, each against the tmax the previous one left.
__device__ __forceinline__ PrimHit intersect_triangle_pre(v3 o, v3 d, float tmin, v3 p1, v3 edge1, v3 edge2) {
    v3 pvec = cross(d, edge2);
    float det = dot(edge1, pvec);
    float inv_det = jl_rcp(det);
    v3 tvec = o - p1;
    float u = dot(tvec, pvec) * inv_det;
    v3 qvec = cross(tvec, edge1);
    float v = dot(d, qvec) * inv_det;
    float t = dot(edge2, qvec) * inv_det;
    PrimHit r;
    r.u = u;
    r.v = v;
    r.t = t;
    r.hit = !((det == 0) | (u < 0 || u > 1) | (v < 0 || u + v > 1) | (t < tmin));
    return r;
}
__device__ __forceinline__ bool tri_hit_before(const PrimHit& p, float tmax) { return p.hit && !(p.t > tmax); }
// triangle records carry the edges p2 - p1, p3 - p1, precomputed on the host (the same floats)
__device__ __forceinline__ PrimHit intersect_triangle(v3 o, v3 d, float tmin, float tmax, v3 p1, v3 p2, v3 p3) {
    return intersect_triangle_e(o, d, tmin, tmax, p1, p2 - p1, p3 - p1);
}
// intersect_quad (src/geometry.jl:238-258); `degenerate` = (p3 == p4), precomputed on the host
__device__ __forceinline__ PrimHit intersect_quad(v3 o, v3 d, float tmin, float tmax, v3 p1, v3 p2, v3 p3, v3 p4,
                                                  bool degenerate) {
    PrimHit i1 = intersect_triangle(o, d, tmin, tmax, p1, p2, p4);
    PrimHit i2 = intersect_triangle(o, d, tmin, tmax, p3, p4, p2);
    if (i2.hit) {
        i2.u = 1 - i2.u;
        i2.v = 1 - i2.v;
    }
    const bool first = degenerate || i1.t < i2.t;
    PrimHit r;
    r.u = first ? i1.u : i2.u;
    r.v = first ? i1.v : i2.v;
    r.t = first ? i1.t : i2.t;
    r.hit = first ? i1.hit : i2.hit;
    return r;
}
__device__ __forceinline__ v3 triangle_normal(v3 p1, v3 p2, v3 p3) { return normalize(cross(p2 - p1, p3 - p1)); }
__device__ __forceinline__ v3 quad_normal(v3 p1, v3 p2, v3 p3, v3 p4) {
    return normalize(triangle_normal(p1, p2, p4) + triangle_normal(p3, p4, p2));
}
// interpolate_triangle / interpolate_quad (src/geometry.jl:275-283)
__device__ __forceinline__ v3 interp_tri(v3 p1, v3 p2, v3 p3, v2 uv) {
    float w = (1 - uv.x) - uv.y;
    return (p1 * w + p2 * uv.x) + p3 * uv.y;
}
__device__ __forceinline__ v2 interp_tri(v2 p1, v2 p2, v2 p3, v2 uv) {
    float w = (1 - uv.x) - uv.y;
    return V2((p1.x * w + p2.x * uv.x) + p3.x * uv.y, (p1.y * w + p2.y * uv.x) + p3.y * uv.y);
}
__device__ __forceinline__ v4 interp_tri(v4 p1, v4 p2, v4 p3, v2 uv) {
    float w = (1 - uv.x) - uv.y;
    return (p1 * w + p2 * uv.x) + p3 * uv.y;
}
template <class T>
__device__ __forceinline__ T interp_quad(T p1, T p2, T p3, T p4, v2 uv) {
    if (uv.x + uv.y <= 1) return interp_tri(p1, p2, p4, uv);
    return interp_tri(p3, p4, p2, V2(1 - uv.x, 1 - uv.y));
}
// triangle_tangents_fromuv (src/geometry.jl:285-316)
__device__ __forceinline__ void triangle_tangents_fromuv(v3 p1, v3 p2, v3 p3, v2 uv1, v2 uv2, v2 uv3, v3& tu, v3& tv) {
    v3 p = p2 - p1, q = p3 - p1;
    v2 s = V2(uv2.x - uv1.x, uv3.x - uv1.x);
    v2 t = V2(uv2.y - uv1.y, uv3.y - uv1.y);
    float div = s.x * t.y - s.y * t.x;
    if (div != 0) {
        tu = V3(t.y * p.x - t.x * q.x, t.y * p.y - t.x * q.y, t.y * p.z - t.x * q.z) / div;
        tv = V3(s.x * q.x - s.y * p.x, s.x * q.y - s.y * p.y, s.x * q.z - s.y * p.z) / div;
    } else {
        tu = V3(1, 0, 0);
        tv = V3(0, 1, 0);
    }
}

}  // namespace jtd
