// jt_kernels.h — the MI355X (gfx950) path-tracing megakernel: every per-lane device function
// and the kernel templates, shared by the translation units that instantiate them.
//
// Replaces trace_samples (Princic-1837592/julia-raytracer src/trace.jl:215-274) and everything
// it calls per (pixel, sample, bounce): trace_sample :584, trace_path :276 / trace_naive :471,
// intersect_scene_bvh / intersect_shape_bvh / intersect_instance_bvh (src/bvh.jl:306-520),
// scene evaluation (src/scene.jl:372-928), shading (src/shading.jl), sampling (src/sampling.jl).
//
// Design: one lane owns one pixel and loops over its samples with path
// regeneration — a lane whose path terminated starts its next sample in the same loop
// iteration in which other lanes continue bouncing, so the wave stays full. Two-level BVH
// traversal is one loop over a unified per-lane stack in LDS (TLAS nodes, instance entries,
// BLAS nodes) so that every lane does one stack pop per iteration whatever level it is at;
// the traversal order (and hence hit tie-breaking) is exactly the reference's. The running
// mean (lerp with w = 1/(s+1), src/trace.jl:631-648) is kept in LDS across samples and
// written once per work unit.
//
// Build: every kernel configuration (JT_LAUNCH_CONFIG) is instantiated in its own translation
// unit (jt_kv.hip, compiled once per configuration) so the kernels compile in parallel; the host
// context (jt_trace.hip) only declares them.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>

#include "jt_bsdf.h"
#include "jt_device.h"

#ifndef JT_STAMPS
#define JT_STAMPS 0
#endif
// pops per node iteration: the LDS-mode FT_NONE kernel (cornellbox) gains with 4 (+1.2 %),
// the HBM-mode mesh kernels lose with 4 or 2 (bathroom1 -4 %, ecosys -1.5 %; gpurun_out/ab_nr)
#ifndef JT_NODE_REPEAT_NONE
#define JT_NODE_REPEAT_NONE 4
#endif
#ifndef JT_NODE_REPEAT
#define JT_NODE_REPEAT 3
#endif
// stack pops of a new query run where it is issued, in the shading phase (most lanes take part)
// rather than in sparser traversal iterations: 2 in the FT_LINL mesh kernels since inline light
// chains (features2 +1.5 %, bathroom1 even; cornellbox -0.4 % with 2,
// profiles/r03_inline/ab_fp_nr.txt), 1 in the others (ecosys lost 7 % with 2)
#ifndef JT_FIRST_POP_NONE
#define JT_FIRST_POP_NONE 1
#endif
#ifndef JT_FIRST_POP
#define JT_FIRST_POP 2
#endif
#ifndef JT_VOTE_P
#define JT_VOTE_P 3
#endif
#ifndef JT_VOTE_N
#define JT_VOTE_N 1
#endif
#ifndef JT_CHILD_PRETEST
#define JT_CHILD_PRETEST 1
#endif
// eval_bsdfcos + sample_bsdfcos_pdf in one branch per material type (jt_bsdf.h eval_bsdfcos_pdf)
#ifndef JT_FUSED_BSDF
#define JT_FUSED_BSDF 1
#endif
#ifndef JT_RAY_FROM_PATH
#define JT_RAY_FROM_PATH 1
#endif

namespace jtk {
using namespace jtd;


// ============================================================================ scene evaluation
// One 16-B row of a record, loaded whole for every lane that reaches it. Without the pin the
// compiler narrows a record load to the fields each path reads, and fields read on different
// paths (or at non-adjacent offsets) become several smaller loads. On gfx950 a gather costs one
// vector-memory wave-instruction whatever its width up to 16 B and whatever the number of active
// lanes (scripts/td_width_bench.hip, scripts/td_lanes_bench.hip), and the HBM-mode kernels are
// bound by exactly those instructions. Only the kernels with scene features pin (!ft_none(F)):
// cornellbox's LDS-mode kernel reads these records from LDS.
template <int F>
__device__ __forceinline__ int4 row16(const void* p) {
    int4 v = *reinterpret_cast<const int4*>(p);
    if (!ft_none(F)) __asm__("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
    return v;
}
// row 3 of DInstShade: material, shape, mat_type, rot_identity
template <int F>
__device__ __forceinline__ int4 inst_ids(const DScene& S, int inst) {
    return row16<F>(reinterpret_cast<const char*>(S.inst_shade + inst) + 48);
}
__device__ __forceinline__ fr3 inst_frame(const DScene& S, int inst) {
    const DInstShade& r = S.inst_shade[inst];
    return frame_from(r.f0, r.f1, r.f2);
}

// eval_position (src/scene.jl:435-476)
template <int F>
__device__ __forceinline__ v3 eval_position(const DScene& S, int inst, int elem, v2 uv) {
    const DInstShade& is = S.inst_shade[inst];
    const int4 sh = row16<F>(S.shapes + inst_ids<F>(S, inst).y);  // DShape row 0: kind, .., idx_base
    const int4 e = S.elems[sh.w + elem];
    const fr3 f = frame_from(is.f0, is.f1, is.f2);
    v3 p1 = xyz(S.pos[e.x]), p2 = xyz(S.pos[e.y]), p3 = xyz(S.pos[e.z]);
    if (!(F & FT_QUAD) || sh.x == KIND_TRI) return transform_point(f, interp_tri(p1, p2, p3, uv));
    return transform_point(f, interp_quad(p1, p2, p3, xyz(S.pos[e.w]), uv));
}
// eval_element_normal (src/scene.jl:578-612): transform_normal(frame, triangle/quad normal),
// with the element normal (and, for an unrotated frame, the whole result) precomputed
// (one load from either array, selected per lane: lanes of both kinds share the instruction)
__device__ __forceinline__ v3 element_normal(const DScene& S, int rot_identity, const fr3& f, int g) {
    const v3 n = xyz((rot_identity ? S.enrm_id : S.enrm)[g]);
    return rot_identity ? n : transform_normal(f, n);
}
template <int F>
__device__ __forceinline__ v3 eval_element_normal(const DScene& S, int inst, int elem) {
    const DInstShade& is = S.inst_shade[inst];
    const int4 ids = inst_ids<F>(S, inst);
    const int4 sh = row16<F>(S.shapes + ids.y);
    return element_normal(S, ids.w, frame_from(is.f0, is.f1, is.f2), sh.w + elem);
}
// eval_normal (src/scene.jl:525-576)
__device__ __forceinline__ v3 eval_normal(const DScene& S, const DShape& sh, const int4& e, const fr3& f, v2 uv) {
    if (sh.nrm_base < 0) {
        v3 p1 = xyz(S.pos[e.x]), p2 = xyz(S.pos[e.y]), p3 = xyz(S.pos[e.z]);
        if (sh.kind == KIND_TRI) return transform_normal(f, triangle_normal(p1, p2, p3));
        return transform_normal(f, quad_normal(p1, p2, p3, xyz(S.pos[e.w])));
    }
    const int b = sh.nrm_base - sh.pos_base;  // normals share vertex ids with positions
    v3 n1 = xyz(S.nrm[e.x + b]), n2 = xyz(S.nrm[e.y + b]), n3 = xyz(S.nrm[e.z + b]);
    if (sh.kind == KIND_TRI) return transform_normal(f, normalize(interp_tri(n1, n2, n3, uv)));
    return transform_normal(f, normalize(interp_quad(n1, n2, n3, xyz(S.nrm[e.w + b]), uv)));
}
// eval_texcoord (src/scene.jl:753-788)
__device__ __forceinline__ v2 eval_texcoord(const DScene& S, const DShape& sh, const int4& e, v2 uv) {
    if (sh.tc_base < 0) return uv;
    const int b = sh.tc_base - sh.pos_base;
    float2 t1 = S.tc[e.x + b], t2 = S.tc[e.y + b], t3 = S.tc[e.z + b];
    if (sh.kind == KIND_TRI) return interp_tri(V2(t1.x, t1.y), V2(t2.x, t2.y), V2(t3.x, t3.y), uv);
    float2 t4 = S.tc[e.w + b];
    return interp_quad(V2(t1.x, t1.y), V2(t2.x, t2.y), V2(t3.x, t3.y), V2(t4.x, t4.y), uv);
}
// eval_color (src/scene.jl:690-720)
__device__ __forceinline__ v4 eval_color(const DScene& S, const DShape& sh, const int4& e, v2 uv) {
    if (sh.col_base < 0) return V4(1, 1, 1, 1);
    const int b = sh.col_base - sh.pos_base;
    float4 c1 = S.col[e.x + b], c2 = S.col[e.y + b], c3 = S.col[e.z + b];
    v4 a = V4(c1.x, c1.y, c1.z, c1.w), bb = V4(c2.x, c2.y, c2.z, c2.w), c = V4(c3.x, c3.y, c3.z, c3.w);
    if (sh.kind == KIND_TRI) return interp_tri(a, bb, c, uv);
    float4 c4 = S.col[e.w + b];
    return interp_quad(a, bb, c, V4(c4.x, c4.y, c4.z, c4.w), uv);
}
// lookup_texture (src/scene.jl:836-849): 8-bit texels decode through exact host-built LUTs
__device__ __forceinline__ v4 lookup_texture(const DScene& S, const DTexture& t, int i, int j, bool as_linear) {
    long long k = t.offset + (long long)j * t.width + i;
    if (t.is_float) {
        float4 c = S.texf[k];
        return V4(c.x, c.y, c.z, c.w);
    }
    uchar4 b = S.texb[k];
    const float* lut = (as_linear && !t.linear) ? S.srgb_lut : S.byte_lut;
    return V4(lut[b.x], lut[b.y], lut[b.z], S.byte_lut[b.w]);
}
// mod1(x, 1.0f0) (Julia base: mod via rem, then 0 -> 1)
__device__ __forceinline__ float jl_mod1(float x) {
    float r = __builtin_fmodf(x, 1.0f);
    float m = r == 0 ? __builtin_copysignf(r, 1.0f) : (r < 0 ? r + 1.0f : r);
    return m == 0 ? 1.0f : m;
}
// two horizontally adjacent 8-bit texels (i, j) and (i + 1, j) in one 8-B load (one vector-memory
// instruction instead of two; texb carries a padding texel past its end)
struct __attribute__((aligned(4))) TexelPair {
    uchar4 a, b;
};
// The two 256-entry texel-decode LUTs (srgb_lut, then byte_lut) in LDS, filled at kernel start
// by the kernels that evaluate textures: a texel's four channel decodes are then LDS reads, not
// four more vector-memory gathers per texel.
static __shared__ float tex_lut[512];
__device__ __forceinline__ v4 decode_texel(uchar4 b, const float* lut) {
    return V4(lut[b.x], lut[b.y], lut[b.z], tex_lut[256 + b.w]);
}
// eval_texture (src/scene.jl:790-834): bilinear, wrap
__device__ __forceinline__ v4 eval_texture(const DScene& S, int tex, v2 uv, bool as_linear) {
    if (tex < 0) return V4(1, 1, 1, 1);
    const DTexture t = S.textures[tex];
    if (t.width == 0 || t.height == 0) return V4(0, 0, 0, 0);
    float s = jl_mod1(uv.x) * (float)t.width;
    if (s < 0) s += (float)t.width;
    float tt = jl_mod1(uv.y) * (float)t.height;
    if (tt < 0) tt += (float)t.height;
    int i = jl_clampi((int)__builtin_truncf(s), 0, t.width - 1);
    int j = jl_clampi((int)__builtin_truncf(tt), 0, t.height - 1);
    int ii = (i + 1) % t.width, jj = (j + 1) % t.height;
    float u = s - (float)i, v = tt - (float)j;
    v4 ta, tb, tc, td;  // texels (i, j), (i, jj), (ii, j), (ii, jj)
    if (t.is_float) {
        ta = lookup_texture(S, t, i, j, as_linear);
        tb = lookup_texture(S, t, i, jj, as_linear);
        tc = lookup_texture(S, t, ii, j, as_linear);
        td = lookup_texture(S, t, ii, jj, as_linear);
    } else {
        const TexelPair r0 = *reinterpret_cast<const TexelPair*>(S.texb + t.offset + (long long)j * t.width + i);
        const TexelPair r1 = *reinterpret_cast<const TexelPair*>(S.texb + t.offset + (long long)jj * t.width + i);
        uchar4 c0 = r0.b, c1 = r1.b;
        if (ii == 0) {  // right edge: the neighbour wraps to column 0
            c0 = S.texb[t.offset + (long long)j * t.width];
            c1 = S.texb[t.offset + (long long)jj * t.width];
        }
        const float* lut = tex_lut + ((as_linear && !t.linear) ? 0 : 256);
        ta = decode_texel(r0.a, lut);
        tb = decode_texel(r1.a, lut);
        tc = decode_texel(c0, lut);
        td = decode_texel(c1, lut);
    }
    v4 a = (ta * (1 - u)) * (1 - v);
    v4 b = (tb * (1 - u)) * v;
    v4 c = (tc * u) * (1 - v);
    v4 d = (td * u) * v;
    return ((a + b) + c) + d;
}
// eval_normalmap (src/scene.jl:722-751) with eval_element_tangents (:851-891)
__device__ __forceinline__ v3 eval_normalmap(const DScene& S, const DShape& sh, const int4& e, const fr3& f,
                                          const DMaterial& m, v2 uv) {
    v3 normal = eval_normal(S, sh, e, f, uv);
    v2 texcoord = eval_texcoord(S, sh, e, uv);
    v4 t4 = eval_texture(S, m.normal_tex, texcoord, false);
    v3 nm = V3(t4.x * 2 - 1, t4.y * 2 - 1, t4.z * 2 - 1);
    v3 tu = V3(0, 0, 0), tv = V3(0, 0, 0);
    if (sh.tc_base >= 0) {
        const int b = sh.tc_base - sh.pos_base;
        float2 a1 = S.tc[e.x + b], a2 = S.tc[e.y + b];
        if (sh.kind == KIND_TRI) {
            float2 a3 = S.tc[e.z + b];
            triangle_tangents_fromuv(xyz(S.pos[e.x]), xyz(S.pos[e.y]), xyz(S.pos[e.z]), V2(a1.x, a1.y),
                                     V2(a2.x, a2.y), V2(a3.x, a3.y), tu, tv);
        } else {  // quad_tangents_fromuv at current_uv = (0, 0): triangle (p1, p2, p4)
            float2 a4 = S.tc[e.w + b];
            triangle_tangents_fromuv(xyz(S.pos[e.x]), xyz(S.pos[e.y]), xyz(S.pos[e.w]), V2(a1.x, a1.y),
                                     V2(a2.x, a2.y), V2(a4.x, a4.y), tu, tv);
        }
        tu = transform_direction(f, tu);
        tv = transform_direction(f, tv);
    }
    v3 f1 = normalize(tu - normal * dot(tu, normal));  // orthonormalize(frame[1], frame[3])
    v3 f2 = normalize(cross(normal, tu));
    bool flip_v = dot(f2, tv) < 0;
    nm = V3(nm.x, nm.y * (flip_v ? 1.0f : -1.0f), nm.z);
    fr3 fr{f1, f2, normal, V3(0, 0, 0)};
    return transform_normal(fr, nm);
}

struct Shading {
    v3 position, normal;
    MatPoint mat;
};

// eval_shading_position + eval_shading_normal + eval_material (src/scene.jl:416-673)
template <int F>
__device__ __forceinline__ void eval_shading(const DScene& S, int inst, int elem, v2 uv, v3 outgoing, Shading& out) {
    const DInstShade is = S.inst_shade[inst];
    const DShape sh = S.shapes[is.shape];
    const int4 e = S.elems[sh.idx_base + elem];
    const fr3 f = frame_from(is.f0, is.f1, is.f2);
    const DMaterial& m = S.materials[is.material];
    v3 p1 = xyz(S.pos[e.x]), p2 = xyz(S.pos[e.y]), p3 = xyz(S.pos[e.z]);
    const bool tri = !(F & FT_QUAD) || sh.kind == KIND_TRI;
    v3 p4 = !tri ? xyz(S.pos[e.w]) : p3;
    // position
    out.position = tri ? transform_point(f, interp_tri(p1, p2, p3, uv))
                       : transform_point(f, interp_quad(p1, p2, p3, p4, uv));
    // shading normal
    const int mtype = (F & FT_MAT) ? m.type : (int)M_MATTE;
    v3 normal;
    if ((F & FT_TEX) && m.normal_tex >= 0) {
        normal = eval_normalmap(S, sh, e, f, m, uv);
    } else if (!(F & FT_ATTR) || sh.nrm_base < 0) {
        normal = element_normal(S, is.rot_identity, f, sh.idx_base + elem);
    } else {
        normal = eval_normal(S, sh, e, f, uv);
    }
    if (mtype != M_REFRACTIVE) normal = dot(normal, outgoing) >= 0 ? normal : -normal;
    out.normal = normal;
    // material point
    MatPoint& p = out.mat;
    const v4 one = V4(1, 1, 1, 1);
    v2 texcoord = (F & FT_ATTR) ? eval_texcoord(S, sh, e, uv) : uv;
    v4 emission_tex = (F & FT_TEX) ? eval_texture(S, m.emission_tex, texcoord, true) : one;
    v4 color_shp = (F & FT_ATTR) ? eval_color(S, sh, e, uv) : one;
    v4 color_tex = (F & FT_TEX) ? eval_texture(S, m.color_tex, texcoord, true) : one;
    v4 roughness_tex = (F & FT_TEX) ? eval_texture(S, m.roughness_tex, texcoord, false) : one;
    v4 scattering_tex = (F & FT_TEX) ? eval_texture(S, m.scattering_tex, texcoord, true) : one;
    p.type = mtype;
    p.emission = V3(m.emission[0], m.emission[1], m.emission[2]) * xyz(emission_tex);
    p.color = (V3(m.color[0], m.color[1], m.color[2]) * xyz(color_tex)) * xyz(color_shp);
    p.opacity = m.opacity * color_tex.w * color_shp.w;
    p.metallic = m.metallic * roughness_tex.z;
    float roughness = m.roughness * roughness_tex.y;
    roughness = roughness * roughness;
    p.ior = m.ior;
    p.scattering = V3(m.scattering[0], m.scattering[1], m.scattering[2]) * xyz(scattering_tex);
    p.scanisotropy = m.scanisotropy;
    p.trdepth = m.trdepth;
    if ((F & FT_VOL) && (mtype == M_REFRACTIVE || mtype == M_VOLUMETRIC || mtype == M_SUBSURFACE)) {
        p.density = V3(-jl_log(jl_clamp(p.color.x, 0.0001f, 1.0f)) / p.trdepth,
                       -jl_log(jl_clamp(p.color.y, 0.0001f, 1.0f)) / p.trdepth,
                       -jl_log(jl_clamp(p.color.z, 0.0001f, 1.0f)) / p.trdepth);
    } else {
        p.density = V3(0, 0, 0);
    }
    if (mtype == M_MATTE || mtype == M_GLTFPBR || mtype == M_GLOSSY) roughness = jl_clamp(roughness, min_roughness, 1.0f);
    else if (mtype == M_VOLUMETRIC) roughness = 0.0f;
    else if (roughness < min_roughness) roughness = 0.0f;
    p.roughness = roughness;
}

// eval_environment (src/scene.jl:893-914)
template <int F>
__device__ __forceinline__ v3 eval_environment(const DScene& S, v3 direction) {
    v3 emission = V3(0, 0, 0);
    if (!(F & FT_ENV)) return emission;  // no environments: the sum is empty
    for (int k = 0; k < S.nenvs; k++) {
        const DEnv& env = S.envs[k];
        v3 wl = transform_direction(frame_from(env.inv), direction);
        v2 tc = V2(jl_atan2(wl.z, wl.x) / (2.0f * pif), jl_acos(jl_clamp(wl.y, -1.0f, 1.0f)) / pif);
        if (tc.x < 0.0f) tc.x = tc.x + 1.0f;
        v4 t = eval_texture(S, env.tex, tc, false);
        emission = emission + V3(env.emission[0], env.emission[1], env.emission[2]) * xyz(t);
    }
    return emission;
}

// ============================================================================ traversal (src/bvh.jl)
// Unified per-lane stack in LDS, entry = type << 30 | snap << 24 | index (24 bits; jt_create
// checks the scene fits). snap (HBM mode): the query's hit count when a pre-tested child was
// pushed (SNAP_NONE: not pre-tested). Layout stack[k * BLOCK + lane]:
// every lane owns one bank (conflict-free ds_read/write_b32 whatever the per-lane depth).
// The LDS part is a ring of RING entries; when a scene's bound exceeds it (OVF), the oldest
// entries spill to a per-lane HBM area (slot blockIdx.x * BLOCK + threadIdx.x of the persistent
// grid: a query never outlives its lane) and come back one at a time when popped.
constexpr int BLOCK = 256;
constexpr unsigned T_TLAS = 0u, T_INST = 1u, T_BLAS = 2u;
constexpr unsigned IDX_MASK = (1u << 24) - 1;
constexpr unsigned SNAP_NONE = 63u << 24;

struct Hit {
    int inst, elem;
    float u, v, t;
    bool hit;
};
struct Counters {  // diagnostic traversal counts (COUNT=1); paths / rays / light queries are per wave
    unsigned nodes, instances, prims, shades;
};

// A resumable BVH query per lane, for intersect_scene_bvh (root = TLAS node 0) and
// intersect_instance_bvh (root = one instance entry). node_step() / prim_step() do one unit of work: one
// node (box test + push), one instance entry (ray to instance space), or ONE primitive test of
// the current leaf (leaf cursor), so every step costs about the same whatever a lane is doing.
// Visit order — children per d[axis] sign (far-first as the reference, or near-first with
// JT_TRAVERSAL_NEAR), a TLAS leaf's instances in order, a BLAS leaf's primitives in order before
// anything else is popped — is the oracle's in either mode, so the closest hit and its
// tie-breaking (t == tmax replaces; only t > tmax rejects) match it.
struct Trav {
    v3 wo, wd, wdinv;  // world-space ray of the query
    v3 lo, ld, ldinv;  // the ray every node test uses: the world ray, or inside a BLAS the ray
                       // in the current instance's space (transform_ray, src/geometry.jl:107)
    float tmax;
    int sp;            // stack entries (all levels)
    int low;           // OVF: entries [low, sp) are in the LDS ring, [0, low) in HBM
    int inst_space;    // lo/ld/ldinv hold an instance-space ray (restore before a TLAS pop)
    int negmask;       // bit a set <=> ld[a] < 0 (the push order of src/bvh.jl:331-341, 424-434),
                       // every bit inverted for JT_TRAVERSAL_NEAR (S.order_flip)
    int cur_inst, cur_kind;
    int prim, nprim;   // leaf cursor: next primitive record, primitives left
    int h_inst, h_elem;  // closest hit so far (instance -1: none); its distance is tmax
    float h_u, h_v;
    int nh;              // bits 0-5: hits accepted so far (every tmax change), saturating at 63;
                         // TIE_SEEN, REF_RERUN (the tie rule below)
    unsigned nxt;        // wide traversal: the child word visited by the next node step (W_EMPTY: pop)
};

// Exact-t ties in the near-first orders (JT_TRAVERSAL_NEAR / WIDE). The reference accepts a hit
// at t == tmax (src/geometry.jl:226, only t > tmax rejects), so among equal-t hits the one it
// tests LAST wins, and which one that is depends on its child order (src/bvh.jl:331-341). A
// near-first query that accepts a hit at exactly its current tmax (TIE_SEEN) is therefore run
// again in the reference's child order (REF_RERUN: the same records, the children visited far
// first; with the wide records that is the binary far-first leaf sequence) and reports that
// query's hit instead: the reference's own tie resolution. Ties are rare (2e-5 of bathroom1's
// queries, none on cornellbox), so the hot path only records them (at an accepted hit), and the
// re-run runs where the query's hit is consumed (rerun_tie). A re-run is the same query: it is
// not counted as a ray or light query again; its node and primitive work is counted (COUNT=1).
#ifndef JT_BAND_STRIP
// tile rows per strip of a band's unit order (1: row-major). Measured against row-major
// (gpurun_out/r05st, r05st2, two runs each): 16 rows cornellbox +2.0 %, features2 +1.1 %, ecosys
// +1.1 %; 8 rows cornellbox +1.3 %, features2 +1.4 %, ecosys +1.1 %, bathroom1 +0.4 %; 4 rows
// and 32 rows in between
#define JT_BAND_STRIP 16
#endif
#ifndef JT_TIE_RERUN
#define JT_TIE_RERUN 1  // 0: ties resolve in the near-first order's own sequence (A/B runs only)
#endif
constexpr int TIE_SEEN = 1 << 8, REF_RERUN = 1 << 9, NH_COUNT = 63;
// the child-order flip of the lane's current query: near-first, unless it is a tie's re-run
__device__ __forceinline__ int query_flip(const DScene& S, const Trav& T) { return (T.nh & REF_RERUN) ? 0 : S.order_flip; }
// a hit accepted at t (t <= tmax): count it (child pre-test snapshots) and note an exact-t tie
__device__ __forceinline__ void hit_count(Trav& T, float t) {
    T.nh = (T.nh + ((T.nh & NH_COUNT) < NH_COUNT ? 1 : 0)) | (JT_TIE_RERUN && t == T.tmax ? TIE_SEEN : 0);
}

__device__ __forceinline__ int neg_mask(v3 d, int flip) {
    return ((d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0)) ^ flip;
}

__device__ __forceinline__ void world_ray(const DScene& S, Trav& T) {
    T.lo = T.wo;
    T.ld = T.wd;
    T.ldinv = T.wdinv;
    T.negmask = neg_mask(T.wd, query_flip(S, T));
    T.inst_space = 0;
}

__device__ __forceinline__ Hit query_hit(const Trav& T) {
    return Hit{T.h_inst, T.h_elem, T.h_u, T.h_v, T.tmax, T.h_inst >= 0};
}

__device__ __forceinline__ bool query_busy(const Trav& T) { return T.sp > 0 || T.nprim > 0; }
// A lane's next step in either traversal: a primitive test (nprim > 0) or a node step (a stack
// entry, or in the wide traversal a pending child word); neither: its query is done (sp 0) or the
// lane has no samples left (sp < 0).
template <bool WIDE>
__device__ __forceinline__ bool wants_node(const Trav& T) {
    return T.nprim == 0 && (T.sp > 0 || (WIDE && T.nxt != W_EMPTY));
}
template <bool WIDE>
__device__ __forceinline__ bool query_done(const Trav& T) {
    return (T.sp | T.nprim) == 0 && (!WIDE || T.nxt == W_EMPTY);
}

__device__ __forceinline__ void query_begin(const DScene& S, Trav& T, v3 o, v3 d, unsigned root, int* stack, int rerun = 0) {
    T.wo = o;
    T.wd = d;
    T.wdinv = V3(jl_rcp(d.x), jl_rcp(d.y), jl_rcp(d.z));  // ray_dinv (src/bvh.jl:322), no guard
    T.lo = o;
    T.ld = d;
    T.ldinv = T.wdinv;
    T.tmax = __builtin_inff();
    T.nh = rerun;
    T.h_inst = -1;
    T.h_elem = -1;
    T.h_u = 0;
    T.h_v = 0;
    T.nprim = 0;
    T.prim = 0;
    T.cur_inst = -1;
    T.cur_kind = KIND_TRI;
    T.inst_space = 0;
    T.negmask = neg_mask(d, rerun ? 0 : S.order_flip);
    stack[0] = (int)root;
    T.sp = 1;
    T.low = 0;
    T.nxt = W_EMPTY;
}
// query_begin of the wide traversal: the root is the first node step's child word (the TLAS
// root record, or an instance leaf of one instance for intersect_instance_bvh); the stack is empty
__device__ __forceinline__ void query_begin_wide(const DScene& S, Trav& T, v3 o, v3 d, unsigned root_word, int rerun = 0) {
    T.wo = o;
    T.wd = d;
    T.wdinv = V3(jl_rcp(d.x), jl_rcp(d.y), jl_rcp(d.z));  // ray_dinv (src/bvh.jl:322), no guard
    T.lo = o;
    T.ld = d;
    T.ldinv = T.wdinv;
    T.tmax = __builtin_inff();
    T.nh = rerun;
    T.h_inst = -1;
    T.h_elem = -1;
    T.h_u = 0;
    T.h_v = 0;
    T.nprim = 0;
    T.prim = 0;
    T.cur_inst = -1;
    T.cur_kind = KIND_TRI;
    T.inst_space = 0;
    T.negmask = neg_mask(d, rerun ? 0 : S.order_flip);
    T.sp = 0;
    T.low = 0;
    T.nxt = root_word;
}
constexpr unsigned WROOT_SCENE = 0u;  // the TLAS root record
__device__ __forceinline__ unsigned wroot_instance(int inst) { return W_LEAF | W_INST | (unsigned)inst; }
// query_begin for either traversal: a closest-hit scene query, or (inst >= 0) the
// intersect_instance_bvh of sample_lights_pdf
template <bool WIDE>
__device__ __forceinline__ void query_start(const DScene& S, Trav& T, v3 o, v3 d, int inst, int* stack, int rerun = 0) {
    if (WIDE) query_begin_wide(S, T, o, d, inst < 0 ? WROOT_SCENE : wroot_instance(inst), rerun);
    else query_begin(S, T, o, d, inst < 0 ? ((T_TLAS << 30) | SNAP_NONE) : ((T_INST << 30) | SNAP_NONE | (unsigned)inst), stack, rerun);
}
// a finished near-first query that saw an exact-t tie: run it again in the reference's child order
// (the same world ray (o, d): every query is started on its path's (st.o, st.d), which do not
// change until its hit is consumed — so T.wo/T.wd stay dead in kernels without instance
// transforms; inst >= 0: the intersect_instance_bvh of that instance). Returns whether the lane
// re-runs (its query is then not done).
// An instance query of a one-leaf BLAS (INST_LEAF_ROOT) tests its leaf's primitives in the same
// order in every child order, so it is never re-run (the oracle's instance_query: the same rule).
constexpr int INST_LEAF_ROOT = 1 << 30;  // in the instance record's w (shape) word
template <bool WIDE>
__device__ __forceinline__ bool rerun_tie(const DScene& S, Trav& T, v3 o, v3 d, int inst, int* stack) {
    if (!JT_TIE_RERUN || (T.nh & (TIE_SEEN | REF_RERUN)) != TIE_SEEN || S.order_flip == 0) return false;
    if (inst >= 0 && (S.inst_blas[inst].w & INST_LEAF_ROOT)) return false;
    query_start<WIDE>(S, T, o, d, inst, stack, REF_RERUN);
    return true;
}

// The current BLAS leaf's next primitive(s), in order (src/bvh.jl:444-484). Triangles go in
// pairs: both tests are computed side by side (the record after the leaf's last one exists: the
// array is padded), then accepted in order, the second against the tmax the first left. A
// second pair runs in the same step when some lane's leaf has more than two left.
// Triangle k of the current leaf and the next one come from one 80-B pair record (host layout:
// the two triangles' components interleaved, 5 loads instead of 6 for two separate records).
// k is 0 or 2.
template <int F>
__device__ __forceinline__ void tri_pair(const DScene& S, Trav& T, int k) {
    const float4* r = S.prims + 5 * (T.prim + (k >> 1));
    const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
    const PrimHit p1 = intersect_triangle_pre(T.lo, T.ld, ray_eps, V3(r0.x, r0.z, r1.x), V3(r1.z, r2.x, r2.z),
                                              V3(r3.x, r3.z, r4.x));
    const PrimHit p2 = intersect_triangle_pre(T.lo, T.ld, ray_eps, V3(r0.y, r0.w, r1.y), V3(r1.w, r2.y, r2.w),
                                              V3(r3.y, r3.w, r4.y));
    if (tri_hit_before(p1, T.tmax)) {
        hit_count(T, p1.t);
        T.h_inst = T.cur_inst;
        T.h_elem = __float_as_int(r4.z);
        T.h_u = p1.u;
        T.h_v = p1.v;
        T.tmax = p1.t;
    }
    if (T.nprim >= k + 2 && tri_hit_before(p2, T.tmax)) {
        hit_count(T, p2.t);
        T.h_inst = T.cur_inst;
        T.h_elem = __float_as_int(r4.w);
        T.h_u = p2.u;
        T.h_v = p2.v;
        T.tmax = p2.t;
    }
}
template <int COUNT, int F>
__device__ __forceinline__ void prim_step(const DScene& S, Trav& T, Counters& cnt) {
    if (!(F & FT_QUAD) || T.cur_kind == KIND_TRI) {
        // a triangle leaf (<= 4 primitives, BVH_MAX_PRIMS, src/bvh.jl:32) is tested within this step
        tri_pair<F>(S, T, 0);
        const bool more = T.nprim > 2;
        if (__builtin_amdgcn_ballot_w64(more)) {
            if (more) tri_pair<F>(S, T, 2);
        }
        const int n = T.nprim < 4 ? T.nprim : 4;
        if (COUNT) cnt.prims += n;
        T.prim += 2;  // pair records (only read again when the leaf had more than four)
        T.nprim -= n;
        return;
    }
    if (COUNT) cnt.prims++;
    const float4* r = S.prims + 4 * T.prim;
    const float4 a = r[0], b = r[1], c = r[2], d = r[3];
    const PrimHit p = intersect_quad(T.lo, T.ld, ray_eps, T.tmax, xyz(a), xyz(b), xyz(c), xyz(d), d.w != 0.0f);
    if (p.hit) {
        hit_count(T, p.t);
        T.h_inst = T.cur_inst;
        T.h_elem = __float_as_int(a.w);
        T.h_u = p.u;
        T.h_v = p.v;
        T.tmax = p.t;
    }
    T.prim += 1;
    T.nprim -= 1;
}

template <int RING, bool OVF>
__device__ __forceinline__ void st_push(const DScene& S, Trav& T, int* stack, int pixel, unsigned e) {
    if (OVF) {
        if (T.sp - T.low == S.ring) {  // ring full: the oldest entry moves to HBM
            S.ovf[(size_t)pixel * S.ovf_stride + T.low] = stack[(T.low & (S.ring - 1)) * BLOCK];
            T.low += 1;
        }
        stack[(T.sp & (S.ring - 1)) * BLOCK] = (int)e;
    } else {
        stack[T.sp * BLOCK] = (int)e;
    }
    T.sp += 1;
}
template <int RING, bool OVF>
__device__ __forceinline__ unsigned st_pop(const DScene& S, Trav& T, const int* stack, int pixel) {
    T.sp -= 1;
    if (OVF) {
        // the ring slot is read unconditionally (its address is always valid; a relaxed atomic
        // load, which the compiler cannot merge with the HBM load) and the HBM entry only below
        // the ring: written as a choice of the two addresses, the compiler made every pop one
        // flat load waiting on both memory counters
        const unsigned r = (unsigned)__hip_atomic_load(stack + (T.sp & (S.ring - 1)) * BLOCK, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_WORKGROUP);
        if (T.sp < T.low) {  // below the ring: this entry was spilled
            T.low = T.sp;
            return (unsigned)S.ovf[(size_t)pixel * S.ovf_stride + T.sp];
        }
        return r;
    }
    return (unsigned)stack[T.sp * BLOCK];
}

// Pop one stack entry: an instance entry or a TLAS/BLAS node. An instance visit and the box
// test of its BLAS root are one step: the reference's instance visit pushes nothing but the
// root (src/bvh.jl:345-351, 502-506), which is then the very next pop, so testing it in the same
// step visits the same nodes in the same order.
template <int RING, bool OVF, int COUNT, bool NCACHE, int F>
__device__ __forceinline__ void node_step(const DScene& S, Trav& T, int* stack, int pixel, Counters& cnt) {
    // without FT_XFORM every instance ray is the world ray: no transform, no space switch
    constexpr bool XF = (F & FT_XFORM) != 0;
    const unsigned e = st_pop<RING, OVF>(S, T, stack, pixel);
    unsigned type = e >> 30, idx = e & IDX_MASK;
    if (type == T_INST) {  // instance visit: inverse(frame, true) precomputed (src/bvh.jl:345,502)
        if (COUNT) cnt.instances++;
        const int4 ib = S.inst_blas[idx];  // blas_root, identity, kind, shape | leaf root (one load: x, y adjacent)
        if (!XF || ib.y) {
            // inverse(identity) is exactly the identity: transform_ray returns the ray bit for bit
            if (XF && T.inst_space) world_ray(S, T);
        } else {
            const DInstTrav it = S.inst_trav[idx];
            const fr3 inv = frame_from(it.i0, it.i1, it.i2);
            T.lo = transform_point(inv, T.wo);
            T.ld = transform_vector(inv, T.wd);
            T.ldinv = V3(jl_rcp(T.ld.x), jl_rcp(T.ld.y), jl_rcp(T.ld.z));
            T.negmask = neg_mask(T.ld, query_flip(S, T));
            T.inst_space = 1;
        }
        T.cur_inst = (int)idx;
        T.cur_kind = ib.z;
        type = T_BLAS;
        idx = (unsigned)ib.x;
    } else if (XF && type == T_TLAS && T.inst_space) {
        world_ray(S, T);  // back from an instance: TLAS nodes test the world ray
    }
    const bool blas = type == T_BLAS;
    if (COUNT) cnt.nodes++;
    // HBM mode: a child pre-tested at its parent with the tmax it still has (no hit since: its
    // snapshot equals the hit count) passes this pop's box test too — same ray, same box, same
    // tmax — so only its start/meta half is loaded
    // The second half (z slab, start/meta) is one load for every lane, the first half only for
    // lanes that test the box: a gather costs one vector-memory wave-instruction whatever the
    // number of active lanes (scripts/td_lanes_bench.hip), so loads shared by both kinds of pop
    // are issued once per step instead of once per kind.
    const unsigned snap = (e >> 24) & 63u;
    float4 nb;
    if (NCACHE) {
        // The second half (z slab, start/meta) is one load for every lane, the first half only
        // for lanes that test the box: a gather costs one vector-memory wave-instruction whatever
        // the number of active lanes (scripts/td_lanes_bench.hip), so a load shared by both kinds
        // of pop is issued once per step instead of once per kind (bathroom1 +3 %, ecosys +2.8 %).
        nb = S.nodes[idx].b;
        // keep it one 16-B load: without this the compiler narrows it to the start/meta half and
        // sinks the z-slab half into the branch below (a second instruction in every mixed step)
        __asm__("" : "+v"(nb.x), "+v"(nb.y), "+v"(nb.z), "+v"(nb.w));
        if (snap == 63u || snap != (unsigned)(T.nh & NH_COUNT))
            if (!intersect_bbox(T.lo, T.ldinv, ray_eps, T.tmax, S.nodes[idx].a, nb)) return;
    } else {  // LDS mode (no pre-test): the whole node, two LDS reads
        const DNode nd = S.nodes[idx];
        if (!intersect_bbox(T.lo, T.ldinv, ray_eps, T.tmax, nd.a, nd.b)) return;
        nb = nd.b;
    }
    const unsigned meta = __float_as_uint(nb.w);
    const int start = __float_as_int(nb.z);
    const int num = (int)(meta & 0xffffu);
    if (meta >> 24) {  // internal: for d[axis] >= 0 push start, start+1 (start+1 pops first)
        const int axis = (int)((meta >> 16) & 0xffu);
        // d[axis] < 0, or (JT_TRAVERSAL_NEAR) d[axis] >= 0: start+1 is pushed first, start pops first
        const bool neg = (T.negmask >> axis) & 1;
        const unsigned tag = type << 30 | SNAP_NONE;
        // c_second is pushed first and popped second, c_first popped first
        const unsigned c_second = (unsigned)(neg ? start + 1 : start), c_first = (unsigned)(neg ? start : start + 1);
        if (JT_CHILD_PRETEST && NCACHE) {
            // HBM mode: test both children (one 64-B pair) when their parent is visited. A child
            // whose box fails now fails when popped too (the slab test is monotone in tmax, which
            // only shrinks): count its pop and skip the push. A pushed child is tested again when
            // popped, with that moment's tmax, exactly as the reference does. (+10 % bathroom1,
            // +14 % ecosys; in LDS mode the extra tests cost more than the pops they save.)
            const DNode n0 = S.nodes[c_second];
            const DNode n1 = S.nodes[c_first];
            const bool k0 = intersect_bbox(T.lo, T.ldinv, ray_eps, T.tmax, n0.a, n0.b);
            const bool k1 = intersect_bbox(T.lo, T.ldinv, ray_eps, T.tmax, n1.a, n1.b);
            if (COUNT) cnt.nodes += (k0 ? 0 : 1) + (k1 ? 0 : 1);
            const unsigned ptag = type << 30 | (unsigned)(T.nh & NH_COUNT) << 24;  // pre-tested at hit count nh
            if (k0) st_push<RING, OVF>(S, T, stack, pixel, ptag | c_second);
            if (k1) st_push<RING, OVF>(S, T, stack, pixel, ptag | c_first);
        } else {
            st_push<RING, OVF>(S, T, stack, pixel, tag | c_second);
            st_push<RING, OVF>(S, T, stack, pixel, tag | c_first);
        }
    } else if (!blas) {  // TLAS leaf: instances start .. start+num-1, in order
        for (int k = num - 1; k >= 0; k--)
            st_push<RING, OVF>(S, T, stack, pixel, (T_INST << 30) | SNAP_NONE | (unsigned)(start + k));
    } else {  // BLAS leaf: its primitives are tested next, in order, before any other pop
        T.prim = start;
        T.nprim = num;

    }
}

// ============================================================================ wide traversal
// JT_TRAVERSAL_WIDE (DWide records, jt_device.h). The children of a record are visited in the
// binary tree's DFS order for the ray: the near pair first by N's axis a0, in each pair the near
// child by a1 / a2 — the same rule as the binary near-first order (S.order_flip folds the order
// into negmask), so leaves are reached in the binary near-first sequence. flips bit 0: the R pair
// first; bit 1 / 2: within L / R the second slot first. Visit index k -> slot:
__device__ __forceinline__ int wide_slot(unsigned flips, int k) {
    const int p = (k >> 1) ^ (int)(flips & 1u);
    return 2 * p + ((k & 1) ^ (int)((flips >> (p ? 2 : 1)) & 1u));
}
__device__ __forceinline__ unsigned wide_word(const uint4& r3, int slot) {
    return slot == 0 ? r3.x : slot == 1 ? r3.y : slot == 2 ? r3.z : r3.w;
}
// dequantised box of slot c (the record's origin + byte * scale, in float) as intersect_bbox's
// (bmin.x, bmax.x, bmin.y, bmax.y), (bmin.z, bmax.z). byte * scale is exact (a byte times a
// normal power of two), so the fused multiply-add rounds once exactly as origin + byte * scale
// does: one v_fma_f32 per plane, the same bits as the host's quantisation check.
__device__ __forceinline__ float deq(float o, unsigned w, int sh, float s) {
    return __builtin_fmaf((float)((w >> sh) & 255u), s, o);
}
__device__ __forceinline__ void wide_box(const float4& r0, const uint4& r1, const uint4& r2, float sx, float sy,
                                         float sz, int c, float4& a, float4& b) {
    const int sh = 8 * c;
    a = make_float4(deq(r0.x, r1.x, sh, sx), deq(r0.x, r1.y, sh, sx), deq(r0.y, r1.z, sh, sy), deq(r0.y, r1.w, sh, sy));
    b = make_float4(deq(r0.z, r2.x, sh, sz), deq(r0.z, r2.y, sh, sz), 0.0f, 0.0f);
}
// Stack entries of the wide traversal (32 bits): a group — the children of record `index` still
// to visit (bit 31 clear; bits 28-30 the record's flips for this ray, 24-27 the visit-order mask
// of children whose boxes passed, 0-23 the record) — or an instance range (bit 31 set; bits 24-25
// count - 1, 0-23 the first instance) of a TLAS leaf whose first instance is being visited.
// A child whose box passed is visited even if tmax has shrunk since (no re-test at pop).
// (Every field is written on both paths: as two branches storing to different fields, the
// compiler merged the stores into one through a selected address, and the Trav fields it addressed
// no longer fit in registers — they lived in scratch, stored per node step.)
template <int F>
__device__ __forceinline__ void wide_take(Trav& T, unsigned w) {
    const bool leaf = (w & (W_LEAF | W_INST)) == W_LEAF;  // a BLAS leaf: its primitives are tested next
    T.prim = leaf ? (int)(w & W_START) : T.prim;
    T.nprim = leaf ? (int)((w >> 28) & 3u) + 1 : T.nprim;

    T.nxt = leaf ? T.nxt : w;  // a record, or a TLAS leaf (its first instance is visited by the next step)
}
// one record visit: the up-to-four child boxes against the current ray and tmax; the first passing
// child (visit order) is taken at once, the others are pushed as one group entry
template <int RING, bool OVF, int COUNT, int F>
__device__ __forceinline__ void wide_visit(const DScene& S, Trav& T, int* stack, int pixel, Counters& cnt, unsigned idx) {
    if (COUNT) cnt.nodes++;
    const DWide& rec = S.wnodes[idx];
    const float4 r0 = rec.r0;
    const uint4 r1 = rec.r1, r2 = rec.r2, r3 = rec.r3;
    const unsigned meta = __float_as_uint(r0.w);
    const float sx = __uint_as_float((meta & 255u) << 23), sy = __uint_as_float(((meta >> 8) & 255u) << 23),
                sz = __uint_as_float(((meta >> 16) & 255u) << 23);
    unsigned hits = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        float4 a, b;
        wide_box(r0, r1, r2, sx, sy, sz, c, a, b);
        const bool pass = intersect_bbox(T.lo, T.ldinv, ray_eps, T.tmax, a, b);
        if (wide_word(r3, c) != W_EMPTY && pass) hits |= 1u << c;
    }
    if (!hits) return;
    const unsigned ax = meta >> 24;
    const unsigned flips = ((T.negmask >> (ax & 3u)) & 1u ? 0u : 1u) | ((T.negmask >> ((ax >> 2) & 3u)) & 1u ? 0u : 2u) |
                           ((T.negmask >> ((ax >> 4) & 3u)) & 1u ? 0u : 4u);
    unsigned vm = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) vm |= ((hits >> wide_slot(flips, k)) & 1u) << k;
    const int k0 = __builtin_ctz(vm);
    const unsigned rest = vm & (vm - 1u);
    if (rest) st_push<RING, OVF>(S, T, stack, pixel, flips << 28 | rest << 24 | idx);
    wide_take<F>(T, wide_word(r3, wide_slot(flips, k0)));
}
// One node step of the wide traversal: the pending child word, or the next child of the group on
// top of the stack (its word: one 4-B load), or the next instance of a range. An instance visit
// (inverse frame precomputed, src/bvh.jl:345,502) and the visit of its BLAS root record are one
// step, as in the binary traversal.
template <int RING, bool OVF, int COUNT, int F>
__device__ __forceinline__ void node_step_wide(const DScene& S, Trav& T, int* stack, int pixel, Counters& cnt) {
    constexpr bool XF = (F & FT_XFORM) != 0;
    unsigned w = T.nxt;
    if (w == W_EMPTY) {
        const unsigned e = st_pop<RING, OVF>(S, T, stack, pixel);
        const unsigned idx = e & IDX_MASK;
        if (!(e >> 31)) {  // a group: its next child in visit order
            const unsigned m = (e >> 24) & 15u;
            const unsigned rest = m & (m - 1u);
            if (rest) st_push<RING, OVF>(S, T, stack, pixel, (e & ~(15u << 24)) | rest << 24);
            if (XF && T.inst_space && idx < (unsigned)S.tlas_wnodes) world_ray(S, T);  // back in the TLAS
            w = reinterpret_cast<const unsigned*>(S.wnodes + idx)[12 + wide_slot((e >> 28) & 7u, __builtin_ctz(m))];
            if ((w & (W_LEAF | W_INST)) == W_LEAF) {
                wide_take<F>(T, w);
                return;
            }
        } else {  // the rest of a TLAS leaf's instances
            w = W_LEAF | W_INST | ((e >> 24) & 3u) << 28 | idx;
        }
    } else {
        T.nxt = W_EMPTY;
    }
    if (w & W_LEAF) {  // a TLAS leaf: visit its first instance, keep the others as a range entry
        const unsigned inst = w & W_START, n1 = (w >> 28) & 3u;
        if (n1) st_push<RING, OVF>(S, T, stack, pixel, W_LEAF | (n1 - 1u) << 24 | (inst + 1u));
        if (COUNT) cnt.instances++;
        const int4 ib = S.inst_blas[inst];  // wide BLAS root record, identity, kind, shape | leaf root
        if (!XF || ib.y) {
            if (XF && T.inst_space) world_ray(S, T);
        } else {
            const DInstTrav it = S.inst_trav[inst];
            const fr3 inv = frame_from(it.i0, it.i1, it.i2);
            T.lo = transform_point(inv, T.wo);
            T.ld = transform_vector(inv, T.wd);
            T.ldinv = V3(jl_rcp(T.ld.x), jl_rcp(T.ld.y), jl_rcp(T.ld.z));
            T.negmask = neg_mask(T.ld, query_flip(S, T));
            T.inst_space = 1;
        }
        T.cur_inst = (int)inst;
        T.cur_kind = ib.z;
        w = (unsigned)ib.x;
    }
    wide_visit<RING, OVF, COUNT, F>(S, T, stack, pixel, cnt, w);
}
// a node step in either traversal
template <bool WIDE, int RING, bool OVF, int COUNT, bool NCACHE, int F>
__device__ __forceinline__ void node_step_any(const DScene& S, Trav& T, int* stack, int pixel, Counters& cnt) {
    if (WIDE) node_step_wide<RING, OVF, COUNT, F>(S, T, stack, pixel, cnt);
    else node_step<RING, OVF, COUNT, NCACHE, F>(S, T, stack, pixel, cnt);
}

// ============================================================================ lights (src/trace.jl)
// sample_lights (src/trace.jl:968-1008)
template <int F>
__device__ __forceinline__ v3 sample_lights(const DScene& S, v3 position, float rl, float rel, v2 ruv) {
    const int light_id = sample_uniform(S.nlights, rl);
    const DLight l = S.lights[light_id - 1];
    const float* cdf = S.cdf + l.cdf_offset;
    if (l.instance >= 0) {
        const int element = l.nguide ? sample_discrete_guided(cdf, l.ncdf, rel, S.guide_t + l.guide_offset,
                                                              S.guide_a + l.guide_offset, l.nguide, l.guide_scale)
                                     : sample_discrete(cdf, l.ncdf, rel);
        const DShape sh = S.shapes[S.inst_shade[l.instance].shape];
        v2 uv = (!(F & FT_QUAD) || sh.kind == KIND_TRI) ? sample_triangle(ruv) : ruv;
        v3 lposition = eval_position<F>(S, l.instance, element - 1, uv);
        return normalize(lposition - position);
    }
    if ((F & FT_ENV) && l.environment >= 0) {
        const DEnv& env = S.envs[l.environment];
        const DTexture t = S.textures[env.tex];
        int idx;  // 1-based, used as-is (:990-993)
        if (l.alias_offset >= 0) {
            // alias-table variant (JT_ENV_ALIAS=1): O(1) — column from rel,
            // keep-or-alias coin from ruv.x (an environment sample does not use ruv). It samples
            // the pmf the CDF holds, so env_light_pdf is unchanged, but it maps random numbers to
            // texels differently from upper_bound: statistically equal, not bit-exact.
            const int col = jl_clampi((int)(rel * (float)l.ncdf), 0, l.ncdf - 1);
            const float2 a = S.alias[l.alias_offset + col];
            idx = (ruv.x < a.x ? col : __float_as_int(a.y)) + 1;
        } else {
            idx = l.nguide ? sample_discrete_guided(cdf, l.ncdf, rel, S.guide_t + l.guide_offset,
                                                    S.guide_a + l.guide_offset, l.nguide, l.guide_scale)
                           : sample_discrete(cdf, l.ncdf, rel);
        }
        float u = ((float)(idx % t.width) + 0.5f) / (float)t.width;
        float v = (float)((((double)idx / (double)t.width) + 0.5) / (double)t.height);
        float su, cu, sv, cv;
        jl_sincos(u * 2 * pif, &su, &cu);
        jl_sincos(v * pif, &sv, &cv);
        return transform_direction(frame_from(env.frame), V3(cu * sv, cv, su * sv));
    }
    return V3(0, 0, 0);
}
// env-light term of sample_lights_pdf (src/trace.jl:1045-1079)
__device__ __forceinline__ float env_light_pdf(const DScene& S, const DLight l, v3 direction) {
    const float* cdf = S.cdf + l.cdf_offset;
    const DEnv& env = S.envs[l.environment];
    const DTexture t = S.textures[env.tex];
    v3 wl = transform_direction(frame_from(env.inv), direction);
    v2 tc = V2(jl_atan2(wl.z, wl.x) / (2 * pif), jl_acos(jl_clamp(wl.y, -1.0f, 1.0f)) / pif);
    if (tc.x < 0) tc.x = tc.x + 1;
    int i = jl_clampi((int)__builtin_truncf(tc.x * (float)t.width), 0, t.width - 1);
    int j = jl_clampi((int)__builtin_truncf(tc.y * (float)t.height), 0, t.height - 1);
    float prob = sample_discrete_pdf(cdf, j * t.width + i + 1) / cdf[l.ncdf - 1];
    float angle = (2 * pif / (float)t.width) * (pif / (float)t.height) *
                  jl_sin(pif * ((float)j + 0.5f) / (float)t.height);
    return prob / angle;
}

// ============================================================================ integrator
// trace_path / trace_naive restated as a per-lane state machine. Every iteration of the
// kernel's shading phase issues exactly one BVH query per waiting lane — a closest-hit scene
// query (PH_SCENE) or one intersect_instance_bvh query of sample_lights_pdf (PH_LIGHT) —
// which the traversal phase then advances (node_step / prim_step). Float operations and RNG draws happen
// in exactly the reference's order; only where the lane waits between them changes.
// PH_FINISH: path done (in a light-hit step), sample not yet accumulated
enum : int { PH_SCENE = 0, PH_LIGHT = 1, PH_FINISH = 2 };
// Light-hit steps (trace_body) run in the path-sampler FT_NONE kernel built without FT_LINL:
// matte scenes whose light chains cannot run inline (a light shape BVH of more than one leaf).
// Every other kernel either runs the chains inline (FT_LINL, or DScene::light_inline at run time)
// or, with environments, shades light results in the shading phase.
__host__ __device__ constexpr bool light_steps(int sampler, int F) {
    return sampler == 1 && !(F & FT_ENV) && !(F & FT_LINL);
}
// the scene's light chains run inline: known at compile time (FT_LINL) or checked at run time
__device__ __forceinline__ bool chains_inline(int F, const DScene& S) { return !(F & FT_NOIL) && ((F & FT_LINL) || S.light_inline); }
enum : int { F_HIT = 1, F_VOLUME = 2 };

// The path's small counters share one register (they are read only in the shading code, and as
// separate registers they were spilled and written back every shading phase):
//   bits 0-14 bounce (jt_create rejects bounces > 32766), 15-22 opbounce (<= 129),
//   23-24 flags (F_HIT, F_VOLUME), 25-31 lcount (the light-query chain, < 100).
constexpr unsigned CTL_BOUNCE = 0x7fffu, CTL_OPB = 15, CTL_FLAGS = 23, CTL_LC = 25;
// Parked path state (JT_PARK): the radiance sum, the light chain's shading position and the
// nocaustics roughness bound are read only in the shading code, so they live in LDS slots of
// the lane (pk[k * BLOCK], after the running means) instead of registers kept live across the
// traversal loop — where the compiler spilled them to scratch (written back every shading phase).
#ifndef JT_PARK
#define JT_PARK 1
#endif
// pb (sample_bsdfcos_pdf of the bounce) is read once, after the bounce's whole light chain: in
// the FT_LINL mesh kernels the chain runs inline, and a register kept live across it was spilled
// and written back to scratch every shading phase (features2: 9.1 GB of WRITE per launch)
#ifndef JT_PARK_PB
#define JT_PARK_PB 1
#endif
constexpr int PARK_SLOTS = 7 + (JT_PARK_PB ? 1 : 0);  // radiance xyz, max_roughness, lq xyz, pb
// slots: [0, 3) radiance, 3 max_roughness, [4, 7) lq, 7 pb. The mesh kernels park (features2 +6 %,
// bathroom1 +14 %, ecosys +9 %: their spills fell from 12-28 to 0-7 VGPRs). The FT_NONE kernel
// (cornellbox, 2-8 spilled VGPRs either way) does not: its light-hit steps read the light-chain
// position every few traversal iterations, and parking cost 4-11 % there (profiles/r03_park/).
__host__ __device__ constexpr bool park(int F) { return JT_PARK != 0 && !ft_none(F); }
__host__ __device__ constexpr bool park_lq(int F) { return park(F); }
__host__ __device__ constexpr int park_slots(int F) { return park(F) ? PARK_SLOTS : 0; }
struct Path {
    v3 o, d;                    // pending ray (during PH_LIGHT the light query's: origin / incoming)
    v3 radiance_, weight_;  // during PH_LIGHT weight already holds weight .* f (src/trace.jl:386)
    Rng rng;
    unsigned ctl;  // bounce | opbounce | flags | lcount (CTL_*)
    int phase;
    float max_roughness_;
    float* pk;  // the lane's parked slots (park(F))
    // sample_lights_pdf in flight (src/trace.jl:1010-1084)
    int li;
    template <int F>
    __device__ __forceinline__ v3 radiance() const {
        return park(F) ? V3(pk[0], pk[BLOCK], pk[2 * BLOCK]) : radiance_;
    }
    template <int F>
    __device__ __forceinline__ void set_radiance(v3 v) {
        if (park(F)) {
            pk[0] = v.x;
            pk[BLOCK] = v.y;
            pk[2 * BLOCK] = v.z;
        } else {
            radiance_ = v;
        }
    }
    template <int F>
    __device__ __forceinline__ v3 lq() const { return park_lq(F) ? V3(pk[4 * BLOCK], pk[5 * BLOCK], pk[6 * BLOCK]) : lq_; }
    template <int F>
    __device__ __forceinline__ void set_lq(v3 v) {
        if (park_lq(F)) {
            pk[4 * BLOCK] = v.x;
            pk[5 * BLOCK] = v.y;
            pk[6 * BLOCK] = v.z;
        } else {
            lq_ = v;
        }
    }
    template <int F>
    __device__ __forceinline__ float max_roughness() const { return park(F) ? pk[3 * BLOCK] : max_roughness_; }
    template <int F>
    __device__ __forceinline__ void set_max_roughness(float v) {
        if (park(F)) pk[3 * BLOCK] = v;
        else max_roughness_ = v;
    }
    template <int F>
    __device__ __forceinline__ float pb() const { return park(F) && JT_PARK_PB ? pk[7 * BLOCK] : pb_; }
    template <int F>
    __device__ __forceinline__ void set_pb(float v) {
        if (park(F) && JT_PARK_PB) pk[7 * BLOCK] = v;
        else pb_ = v;
    }
    // the path weight stays in registers (parked in three more LDS slots it cost the texture
    // kernels a workgroup per CU: DESIGN.md §2 Experiments)
    template <int F>
    __device__ __forceinline__ v3 weight() const { return weight_; }
    template <int F>
    __device__ __forceinline__ void set_weight(v3 v) { weight_ = v; }
    __device__ __forceinline__ int bounce() const { return (int)(ctl & CTL_BOUNCE); }
    __device__ __forceinline__ int opbounce() const { return (int)((ctl >> CTL_OPB) & 0xffu); }
    __device__ __forceinline__ bool flag(int f) const { return (ctl >> CTL_FLAGS) & (unsigned)f; }
    __device__ __forceinline__ void set_flag(int f) { ctl |= (unsigned)f << CTL_FLAGS; }
    __device__ __forceinline__ void clear_flag(int f) { ctl &= ~((unsigned)f << CTL_FLAGS); }
    __device__ __forceinline__ int lcount() const { return (int)(ctl >> CTL_LC); }
    v3 lq_;      // during PH_LIGHT: the shading position (st.o holds the light query's origin,
                 // next_position of src/trace.jl:1039, so every query's ray is (st.o, st.d))
    float pb_;   // sample_bsdfcos_pdf / sample_scattering_pdf (pb<F>(): parked in the mesh kernels)
    float pdf, lpdf;
    Volume vol;  // volume_stack[1] (the stack never holds more than one entry)
};

// while bounce < params.bounces: bounce += 1 (src/trace.jl:295-297, 487-489)
__device__ __forceinline__ bool next_bounce(const DParams& P, Path& st) {
    if (st.bounce() >= P.bounces) return true;
    st.ctl += 1u;  // bounce += 1
    st.phase = PH_SCENE;
    return false;
}
// the opacity retry (src/trace.jl:334-339): bounce -= 1, then the loop's bounce += 1, i.e. the
// loop condition tested with bounce - 1 and bounce unchanged
__device__ __forceinline__ bool next_bounce_retry(const DParams& P, Path& st) {
    if (st.bounce() - 1 >= P.bounces) return true;
    st.phase = PH_SCENE;
    return false;
}
// end of a bounce: weight checks and Russian roulette (src/trace.jl:455-465, 557-567)
template <int F>
__device__ __forceinline__ bool after_weight(const DParams& P, Path& st) {
    if (is_zero(st.weight<F>()) || !all_finite(st.weight<F>())) return true;
    if (st.bounce() > 3) {
        float rr_prob = jl_min(0.99f, max3(st.weight<F>()));
        if (rand1f(st.rng) >= rr_prob) return true;
        st.set_weight<F>(st.weight<F>() * (1 / rr_prob));
    }
    return next_bounce(P, st);
}
// walk the light list: environment terms are added in place, an instance light starts its
// query chain; after the last light the one-sample MIS weight is applied (src/trace.jl:386-397)
template <int F>
__device__ __forceinline__ bool light_advance(const DScene& S, const DParams& P, Path& st) {
    for (;;) {
        st.li += 1;
        if (st.li >= S.nlights) {
            st.o = st.lq<F>();  // the next bounce's ray starts at the shading position
            const float pdf = st.pdf * S.light_pick_pdf;  // sample_uniform_pdf(nlights), host-computed
            st.set_weight<F>(st.weight<F>() / (0.5f * st.pb<F>() + 0.5f * pdf));  // (weight .* f) / (...)
            return after_weight<F>(P, st);
        }
        const DLight l = S.lights[st.li];
        if (!(F & FT_NOIL) && l.instance >= 0) {
            st.lpdf = 0.0f;
            st.ctl &= (1u << CTL_LC) - 1u;  // lcount = 0
            st.o = st.lq<F>();  // the first query starts at the shading position
            st.phase = PH_LIGHT;
            return false;
        }
        if ((F & FT_ENV) && l.environment >= 0) st.pdf += env_light_pdf(S, l, st.d);
    }
}
template <int F>
__device__ __forceinline__ bool begin_light_pdf(const DScene& S, const DParams& P, Path& st) {
    st.pdf = 0.0f;
    st.li = -1;
    st.set_lq<F>(st.o);
    return light_advance<F>(S, P, st);
}
// one intersect_instance_bvh result of the instance-light loop (src/trace.jl:1024-1044)
template <int F>
__device__ __forceinline__ bool light_hit(const DScene& S, const DParams& P, Path& st, const Hit& h) {
    if (h.hit) {
        // the light's element record (DLightElem): eval_position + eval_element_normal + the area
        const int4 lh = row16<F>(S.light_hit + st.li);  // instance, first record
        const DInstShade& is = S.inst_shade[lh.x];
        const fr3 f = frame_from(is.f0, is.f1, is.f2);
        const float4* r = S.light_elems + 5 * (lh.y + h.elem);
        const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3];
        const v3 p1 = V3(r0.x, r0.y, r0.z), p2 = V3(r0.w, r1.x, r1.y), p3 = V3(r1.z, r1.w, r2.x);
        const v2 uv = V2(h.u, h.v);
        v3 lposition;
        if (!(F & FT_QUAD) || __float_as_int(r3.z) == KIND_TRI) {
            lposition = transform_point(f, interp_tri(p1, p2, p3, uv));
        } else {
            const float4 r4 = r[4];
            lposition = transform_point(f, interp_quad(p1, p2, p3, V3(r4.x, r4.y, r4.z), uv));
        }
        const v3 en = V3(r2.y, r2.z, r2.w);
        v3 lnormal = __float_as_int(r3.y) ? en : transform_normal(f, en);
        const float area = r3.x;
        v3 dd = lposition - st.lq<F>();
        st.lpdf += dot(dd, dd) / (__builtin_fabsf(dot(lnormal, st.d)) * area);
        st.o = lposition + st.d * 0.001f;
        st.ctl += 1u << CTL_LC;  // lcount += 1 (< 100: fits its 7 bits)
        if (st.lcount() < 100) return false;
    }
    st.pdf += st.lpdf;
    return light_advance<F>(S, P, st);
}

// The light chain of sample_lights_pdf run inline (DScene::light_inline: every instance light's
// shape BVH is one leaf): each intersect_instance_bvh (src/bvh.jl:493-520) is the instance visit
// with its root box test (node_step) and the leaf's primitives (prim_step), then light_hit, until
// the chain leaves its instance lights. The same functions and the same per-lane order as through
// the traversal loop, so results and counters are unchanged; only where the lane runs them moves:
// here, where most of the wave's lanes run their chains side by side, instead of one-prim-step
// queries and light-hit steps of a few lanes inside the traversal phase. Returns light_hit's
// "path done"; otherwise st.phase is PH_SCENE (the next bounce's scene query).
template <bool WIDE, int RING, bool OVF, int COUNT, bool NCACHE, int F, class CountLq>
__device__ __forceinline__ bool light_chain(const DScene& S, const DParams& P, Path& st, Trav& T, int* stack, int pixel,
                                            Counters& cnt, CountLq count_lq) {
    do {
        count_lq();
        const int inst = S.lights[st.li].instance;
        query_start<WIDE>(S, T, st.o, st.d, inst, stack);
        // No tie re-run is needed here: a one-leaf BLAS has no child order (INST_LEAF_ROOT). The
        // FT_MESH kernel (bathroom1) keeps the re-run loop anyway, never taken: its compiled
        // layout is 4 % faster with it, features2's kernel 1.5 % slower (gpurun_out/r05v)
        constexpr bool RERUN_LOOP = (F & ~FT_LINL) == (FT_TEX | FT_ATTR | FT_MAT | FT_OPAC | FT_XFORM);  // FT_MESH
        do {
            node_step_any<WIDE, RING, OVF, COUNT, NCACHE, F>(S, T, stack, pixel, cnt);  // instance + its one-leaf root
            while (T.nprim > 0) prim_step<COUNT, F>(S, T, cnt);
        } while (RERUN_LOOP && rerun_tie<WIDE>(S, T, st.o, st.d, inst, stack));
        if (light_hit<F>(S, P, st, query_hit(T))) return true;
    } while (st.phase == PH_LIGHT);
    return false;
}

// trace_path's bounce body after the closest-hit query (src/trace.jl:298-453)
// The albedo/normal running means (src/trace.jl:635-636) are updated as soon as the bounce-0
// surface is accepted — their targets are final at that point — so they are not path state.
// Per-lane running means of the lane's pixel, kept in LDS for the whole launch (a lane owns
// its pixel for all its samples): acc[k * BLOCK], k = 0..3 image rgba, 4..6 albedo, 7..9
// normal, 10 hit count of this launch (int). Loaded from / stored to HBM once per launch; the
// per-sample lerps are the same float operations as a read-modify-write of the HBM buffers.
// JT_LANE_LDS: 11 the lane's current sample (int), 12 its running-mean weight 1/(n+1) — per-sample
// state parked in LDS instead of registers kept live (and spilled) across the traversal loop.
#ifndef JT_LANE_LDS
#define JT_LANE_LDS 1
#endif
// The mesh kernels gain (features2 +7 %, bathroom1 +1 %, ecosys +0.6 %). The FT_NONE kernels
// keep only the sample index (12 slots, the weight is recomputed from it): with 13 slots
// cornellbox's LDS-mode kernel no longer fit 5 workgroups per CU (-9 %); with 12 it does, and
// its spills drop from 37 to 23 VGPRs (scratch 112 -> 80 B/lane, spill write-back 36.3 -> 22.6
// GB per launch, +0.5 %; gpurun_out/ab_ll, s8).
#ifndef JT_LANE_LDS_NONE
#define JT_LANE_LDS_NONE 1
#endif
__host__ __device__ constexpr bool lane_lds(int F) { return JT_LANE_LDS && (!ft_none(F) || JT_LANE_LDS_NONE); }
constexpr int ACC_SLOTS = (JT_LANE_LDS ? 13 : 11) + (JT_PARK ? PARK_SLOTS : 0);  // the host sizes LDS for the larger layout
// Lane-LDS slots: [11] the lane's sample index, [12] its running-mean weight. The FT_NONE
// kernels (JT_LANE_LDS_NONE) recompute the weight from the sample index instead of storing it:
// with 12 slots cornellbox's LDS-mode workgroup still fits 5 per CU.
__host__ __device__ constexpr int acc_base_slots(int F) { return lane_lds(F) ? (ft_none(F) ? 12 : 13) : 11; }
// + the parked path state (JT_PARK, Path::pk = acc + acc_base_slots(F) * BLOCK)
__host__ __device__ constexpr int acc_slots(int F) { return acc_base_slots(F) + park_slots(F); }
struct Aov {
    float* acc;
    float w_;    // !lane_lds(F)
    int first_;  // params.first (the weight's sample offset)
    int lk_;     // params.lk (log2 of the sample streams)
    // the running-mean weight of the lane's current sample within its stream (stream_weight)
    template <int F>
    __device__ __forceinline__ float w() const {
        if (!lane_lds(F)) return w_;
        if (ft_none(F)) return 1.0f / (float)(((reinterpret_cast<const int*>(acc)[11 * BLOCK] - first_) >> lk_) + 1);
        return acc[12 * BLOCK];
    }
};
template <int F>
__device__ __forceinline__ void aov_update(const Aov& a, v3 ta, v3 tn) {
    const float aw = a.w<F>();
    const float omw = 1 - aw;
    float* p = a.acc;
    p[4 * BLOCK] = p[4 * BLOCK] * omw + ta.x * aw;
    p[5 * BLOCK] = p[5 * BLOCK] * omw + ta.y * aw;
    p[6 * BLOCK] = p[6 * BLOCK] * omw + ta.z * aw;
    p[7 * BLOCK] = p[7 * BLOCK] * omw + tn.x * aw;
    p[8 * BLOCK] = p[8 * BLOCK] * omw + tn.y * aw;
    p[9 * BLOCK] = p[9 * BLOCK] * omw + tn.z * aw;
}

template <int F, class AovT>
__device__ __forceinline__ bool path_hit(const DScene& S, const DParams& P, Path& st, Hit isec, const AovT& aov,
                                         unsigned& shades) {
    if (!isec.hit) {
        if (st.bounce() > 0 || !P.envhidden)
            st.set_radiance<F>(st.radiance<F>() + st.weight<F>() * eval_environment<F>(S, st.d));
        return true;
    }
    bool in_volume = false;
    if ((F & FT_VOL) && st.flag(F_VOLUME)) {  // :307-326 (volumes need a volume material)
        float rl = rand1f(st.rng), rd = rand1f(st.rng);
        float distance = sample_transmittance(st.vol.density, isec.t, rl, rd);
        v3 tr = eval_transmittance(st.vol.density, distance);
        float tp = sample_transmittance_pdf(st.vol.density, distance, isec.t);
        st.set_weight<F>((st.weight<F>() * tr) / tp);
        in_volume = distance < isec.t;
        isec.t = distance;
    }
    if (!in_volume) {  // surface (:328-423)
        v3 outgoing = -st.d;
        Shading sh;
        eval_shading<F>(S, isec.inst, isec.elem, V2(isec.u, isec.v), outgoing, sh);
        shades++;
        if (P.nocaustics) {
            st.set_max_roughness<F>(jl_max(sh.mat.roughness, st.max_roughness<F>()));
            sh.mat.roughness = st.max_roughness<F>();
        }
        if ((F & FT_OPAC) && sh.mat.opacity < 1 && rand1f(st.rng) >= sh.mat.opacity) {
            if (st.opbounce() > 128) return true;
            st.ctl += 1u << CTL_OPB;  // opbounce += 1 (<= 129)
            st.o = sh.position + st.d * 0.01f;
            return next_bounce_retry(P, st);  // bounce -= 1, then the loop's bounce += 1
        }
        if (st.bounce() == 0) {
            st.set_flag(F_HIT);
            aov_update<F>(aov, sh.mat.color, sh.normal);
        }
        st.set_radiance<F>(st.radiance<F>() + st.weight<F>() * (dot(sh.normal, outgoing) >= 0 ? sh.mat.emission : V3(0, 0, 0)));
        v3 incoming;
        const bool delta = is_delta(sh.mat);
        if (!delta) {
            if (rand1f(st.rng) < 0.5f) {
                float rnl = rand1f(st.rng);
                v2 rn = rand2f(st.rng);
                incoming = sample_bsdfcos<F>(sh.mat, sh.normal, outgoing, rnl, rn);
            } else {
                float rl = rand1f(st.rng), rel = rand1f(st.rng);
                v2 ruv = rand2f(st.rng);
                incoming = sample_lights<F>(S, sh.position, rl, rel, ruv);
            }
            if (is_zero(incoming)) return true;
#if JT_FUSED_BSDF
            v3 fb;
            float pbv;
            eval_bsdfcos_pdf<F>(sh.mat, sh.normal, outgoing, incoming, fb, pbv);
            st.set_weight<F>(st.weight<F>() * fb);
            st.set_pb<F>(pbv);
#else
            st.set_weight<F>(st.weight<F>() * eval_bsdfcos<F>(sh.mat, sh.normal, outgoing, incoming));
            st.set_pb<F>(sample_bsdfcos_pdf<F>(sh.mat, sh.normal, outgoing, incoming));
#endif
        } else {
            float rnl = rand1f(st.rng);
            incoming = sample_delta<F>(sh.mat, sh.normal, outgoing, rnl);
            v3 f = eval_delta<F>(sh.mat, sh.normal, outgoing, incoming);
            float pd = sample_delta_pdf<F>(sh.mat, sh.normal, outgoing, incoming);
            st.set_weight<F>((st.weight<F>() * f) / pd);
        }
        // volume stack push/pop (:405-421); independent of the weight update it follows
        const int mtype = sh.mat.type;
        if ((F & FT_VOL) && (mtype == M_REFRACTIVE || mtype == M_VOLUMETRIC || mtype == M_SUBSURFACE) &&
            dot(sh.normal, outgoing) * dot(sh.normal, incoming) < 0) {
            if (!st.flag(F_VOLUME)) {
                st.set_flag(F_VOLUME);  // eval_material again: only the volume fields are kept
                st.vol.density = sh.mat.density;
                st.vol.scattering = sh.mat.scattering;
                st.vol.scanisotropy = sh.mat.scanisotropy;
            } else {
                st.clear_flag(F_VOLUME);
            }
        }
        st.o = sh.position;
        st.d = incoming;
        return delta ? after_weight<F>(P, st) : begin_light_pdf<F>(S, P, st);
    }
    // volume scattering (:424-453)
    v3 outgoing = -st.d;
    v3 position = st.o + st.d * isec.t;
    v3 incoming;
    if (rand1f(st.rng) < 0.5f) {
        (void)rand1f(st.rng);  // rnl: drawn, unused by sample_scattering
        v2 rn = rand2f(st.rng);
        incoming = sample_scattering(st.vol, outgoing, rn);
    } else {
        float rl = rand1f(st.rng), rel = rand1f(st.rng);
        v2 ruv = rand2f(st.rng);
        incoming = sample_lights<F>(S, position, rl, rel, ruv);
    }
    if (is_zero(incoming)) return true;
    st.set_weight<F>(st.weight<F>() * eval_scattering(st.vol, outgoing, incoming));
    st.set_pb<F>(sample_scattering_pdf(st.vol, outgoing, incoming));
    st.o = position;
    st.d = incoming;
    return begin_light_pdf<F>(S, P, st);
}

// trace_naive's bounce body after the closest-hit query (src/trace.jl:490-569)
template <int F, class AovT>
__device__ __forceinline__ bool naive_hit(const DScene& S, const DParams& P, Path& st, Hit isec, const AovT& aov,
                                          unsigned& shades) {
    if (!isec.hit) {
        if (st.bounce() > 0 || !P.envhidden)
            st.set_radiance<F>(st.radiance<F>() + st.weight<F>() * eval_environment<F>(S, st.d));
        return true;
    }
    v3 outgoing = -st.d;
    Shading sh;
    eval_shading<F>(S, isec.inst, isec.elem, V2(isec.u, isec.v), outgoing, sh);
    shades++;
    if ((F & FT_OPAC) && sh.mat.opacity < 1 && rand1f(st.rng) >= sh.mat.opacity) {
        if (st.opbounce() > 128) return true;
        st.ctl += 1u << CTL_OPB;  // opbounce += 1 (<= 129)
        st.o = sh.position + st.d * 0.01f;
        return next_bounce_retry(P, st);  // bounce -= 1, then the loop's bounce += 1
    }
    if (st.bounce() == 0) {
        st.set_flag(F_HIT);
        aov_update<F>(aov, sh.mat.color, sh.normal);
    }
    st.set_radiance<F>(st.radiance<F>() + st.weight<F>() * (dot(sh.normal, outgoing) >= 0 ? sh.mat.emission : V3(0, 0, 0)));
    v3 incoming, f;
    float p;
    if (sh.mat.roughness != 0) {
        float rnl = rand1f(st.rng);
        v2 rn = rand2f(st.rng);
        incoming = sample_bsdfcos<F>(sh.mat, sh.normal, outgoing, rnl, rn);
        if (is_zero(incoming)) return true;
#if JT_FUSED_BSDF
        eval_bsdfcos_pdf<F>(sh.mat, sh.normal, outgoing, incoming, f, p);
#else
        f = eval_bsdfcos<F>(sh.mat, sh.normal, outgoing, incoming);
        p = sample_bsdfcos_pdf<F>(sh.mat, sh.normal, outgoing, incoming);
#endif
    } else {
        float rnl = rand1f(st.rng);
        incoming = sample_delta<F>(sh.mat, sh.normal, outgoing, rnl);
        if (is_zero(incoming)) return true;
        f = eval_delta<F>(sh.mat, sh.normal, outgoing, incoming);
        p = sample_delta_pdf<F>(sh.mat, sh.normal, outgoing, incoming);
    }
    st.set_weight<F>((st.weight<F>() * f) / p);
    st.o = sh.position;
    st.d = incoming;
    return after_weight<F>(P, st);
}

// eval_camera (src/scene.jl:372-411)
__device__ __forceinline__ void eval_camera(const DCamera& cam, v2 image_uv, v2 lens_uv, v3& ro, v3& rd) {
    const fr3 frame = frame_from(cam.frame);
    const v2 film = V2(cam.film_x, cam.film_y);
    if (!cam.orthographic) {
        v3 q = V3(film.x * (0.5f - image_uv.x), film.y * (image_uv.y - 0.5f), cam.lens);
        v3 dc = -normalize(q);
        v3 e = V3(lens_uv.x * cam.aperture / 2, lens_uv.y * cam.aperture / 2, 0);
        v3 p = (dc * cam.focus) / __builtin_fabsf(dc.z);
        v3 d = normalize(p - e);
        ro = transform_point(frame, e);
        rd = transform_direction(frame, d);
    } else {
        float scale = 1 / cam.lens;
        v3 q = V3(film.x * (0.5f - image_uv.x) * scale, film.y * (image_uv.y - 0.5f) * scale, cam.lens);
        v3 e = V3(-q.x, -q.y, 0) + V3(lens_uv.x * cam.aperture / 2, lens_uv.y * cam.aperture / 2, 0);
        v3 p = V3(-q.x, -q.y, -cam.focus);
        v3 d = normalize(p - e);
        ro = transform_point(frame, e);
        rd = transform_direction(frame, d);
    }
}

// trace_sample prologue (src/trace.jl:597-608): 4 draws, camera ray (sample_camera :651-674)
template <int F>
__device__ __forceinline__ void start_path(const DParams& P, int i, int j, int pixel, int sample, Path& st) {
    st.rng = rng_init(P.seed, pixel, sample);
    v2 puv = rand2f(st.rng);
    v2 luv = rand2f(st.rng);
    v2 uv;
    if (!P.tentfilter) {
        uv = V2(((float)i + puv.x) / (float)P.width, ((float)j + puv.y) / (float)P.height);
    } else {
        const float width = 2.0f, offset = 0.5f;
        v2 fuv = V2(width * (puv.x < 0.5f ? __builtin_sqrtf(2 * puv.x) - 1 : 1 - __builtin_sqrtf(2 - 2 * puv.x)) + offset,
                    width * (puv.y < 0.5f ? __builtin_sqrtf(2 * puv.y) - 1 : 1 - __builtin_sqrtf(2 - 2 * puv.y)) + offset);
        uv = V2(((float)i + fuv.x) / (float)P.width, ((float)j + fuv.y) / (float)P.height);
    }
    eval_camera(P.cam, uv, P.cam.pinhole ? sample_disk_signs(luv) : sample_disk(luv), st.o, st.d);
    st.set_radiance<F>(V3(0, 0, 0));
    st.set_weight<F>(V3(1, 1, 1));
    st.set_max_roughness<F>(0.0f);
    st.ctl = 0u;  // bounce 0 (the first loop iteration: -1 + 1; bounces >= 0 always enters), no flags
    st.phase = PH_SCENE;
}

// active lanes of a ballot, as a 32-bit scalar (keeps the comparisons of counts on the SALU)
__device__ __forceinline__ int lane_count(unsigned long long m) {
    return __builtin_popcount((unsigned)m) + __builtin_popcount((unsigned)(m >> 32));
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

struct DAccum {
    float4* image;
    float4* albedo;
    float4* normal;
    long long* hits;
    unsigned long long* counters;  // 7 x u64: paths rays light_queries nodes instances prims shades;
                                   // [8..31]: the stamps build's per-phase clocks (JT_STAMPS)
    unsigned* work;                // unit counters of the launch, one per XCD band at work[16 b]
                                   // (zeroed before each launch)
    // sample-stream means (P.lk > 0): stream j of a pixel at [j * nslot + slot], slot = the pixel's
    // place in the launch's tiles (item_slot: launch tile u * 64 + pixel of the tile), so a tile
    // share stores only its own pixels; image RGBA, albedo xyz + the stream's hit count (int bits
    // in w), normal xyz
    float4* part_img;
    float4* part_alb;
    float4* part_nrm;
    int nslot;  // launch tiles x 64 (the allocation's slots per stream)
};

// The kernels' argument layout (trace_kernel, trace_kernel_lds: by-value arguments in this order,
// each at its natural alignment, as the AMDGPU kernarg segment lays them out).
struct KArgs {
    DScene S;
    DParams P;
    int s_begin, s_end;
    DAccum A;
};
// JT_KARG_RELOAD: the launch's sample range and accumulator pointers are read from the kernel
// argument segment (a scalar load through the kernarg pointer, laundered so it is not hoisted)
// where they are used — at a work unit's fetch, an item's start and end — instead of being kept in
// SGPRs across the path loop, where the register allocator spilled them to VGPR lanes and reloaded
// them with v_readlane (a VALU instruction and a hazard wait each) in every shading phase.
// Measured against keeping them (two runs each, interleaved, profiles/r06_ab/karg_reload_r06karg.txt):
// cornellbox +3.1 %, bathroom1 1920x1080x64 +1.8 %, ecosys 3840x2160x8 +11 %, features2 -1.5 % (its
// kernel's VGPR spills rose from 3 to 6), so the FT_MESH_ENV_QUAD kernel keeps them in registers.
#ifndef JT_KARG_RELOAD
#define JT_KARG_RELOAD 1
#endif
template <int F>
__host__ __device__ constexpr bool karg_reload() {
    // FT_MESH_ENV_QUAD (below): textures, attributes, materials, opacity, transforms, environments, quads
    return JT_KARG_RELOAD && (F & ~(FT_LINL | FT_NOIL)) != (FT_TEX | FT_ATTR | FT_MAT | FT_OPAC | FT_XFORM | FT_ENV | FT_QUAD);
}
template <class T>
__device__ __forceinline__ T karg(size_t off) {
    typedef __attribute__((address_space(4))) const char* kptr;
    kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const __attribute__((address_space(4))) T*)(p + off);
}
// JT_KARG_SCENE (HBM-mode kernels, whose scene is the kernel argument itself): the shading phase
// reads the scene's fields through the kernarg segment too (one scalar load per field used there,
// re-issued every phase), instead of keeping every pointer the shading code needs live in SGPRs
// across the traversal loop. Measured (two runs each, interleaved, profiles/r06_ab/
// karg_scene_r06ks.txt): features2 1920x1080x64 +3.7 %, materials2 +1.4 %, features1 +0.9 %,
// ecosys +0.8 %, cornellbox (LDS mode: not used) even; bathroom1 -2.1 %, so the FT_MESH kernel
// keeps its scene in registers.
#ifndef JT_KARG_SCENE
#define JT_KARG_SCENE 1
#endif
template <bool NCACHE, int F>
__host__ __device__ constexpr bool karg_scene() {
    // FT_MESH (below): textures, attributes, materials, opacity, transforms
    return NCACHE && JT_KARG_SCENE && (F & ~(FT_LINL | FT_NOIL)) != (FT_TEX | FT_ATTR | FT_MAT | FT_OPAC | FT_XFORM);
}
template <bool FROM_KARG>
__device__ __forceinline__ const DScene& shade_scene(const DScene& S) {
    if constexpr (FROM_KARG) {
        typedef __attribute__((address_space(4))) const char* kptr;
        kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(p));
        return *(const DScene*)(const __attribute__((address_space(4))) DScene*)(p + offsetof(KArgs, S));
    } else {
        return S;
    }
}
// JT_KARG_PARAMS: the sample start and the shading phase read the render parameters (camera,
// bounces, clamp, flags) through the kernarg segment too (the cornellbox kernel's SGPR spills
// 36 -> 16, VGPR spills 1 -> 0). Two runs each (profiles/r06_ab/karg_params_r06kp.txt): cornellbox
// +0.7 %, ecosys +1.0 %, features2 +0.9 %, materials2 +0.2 %; config 1's naive kernel -0.8 % and
// bathroom1 -0.5 %, so the path-sampler kernels other than FT_MESH use it
#ifndef JT_KARG_PARAMS
#define JT_KARG_PARAMS 1
#endif
template <int SAMPLER, int F>
__host__ __device__ constexpr bool karg_params_on() {
    return JT_KARG_PARAMS && SAMPLER == 1 && (F & ~(FT_LINL | FT_NOIL)) != (FT_TEX | FT_ATTR | FT_MAT | FT_OPAC | FT_XFORM);
}
template <bool FROM_KARG>
__device__ __forceinline__ const DParams& karg_params(const DParams& P) {
    if constexpr (FROM_KARG) {
        typedef __attribute__((address_space(4))) const char* kptr;
        kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(p));
        return *(const DParams*)(const __attribute__((address_space(4))) DParams*)(p + offsetof(KArgs, P));
    } else {
        return P;
    }
}
// JT_KARG_SCENE_LDS: the same in the LDS-mode kernels, whose scene is the blob view of the kernel
// argument (blob_scene): the shading phase rebuilds the view from the kernarg segment (the
// cornellbox kernel's SGPR spills 53 -> 36; two runs each, profiles/r06_ab/karg_scene_lds_r06ksl.txt:
// cornellbox +0.35 %, its 1/8 share +0.3 %, config 1 even)
#ifndef JT_KARG_SCENE_LDS
#define JT_KARG_SCENE_LDS 1
#endif
__device__ __forceinline__ DScene blob_scene(const DScene& S, const uint4* blob);
__host__ __device__ constexpr size_t lds_stack_bytes(bool ovf, int ring, int need);
template <bool NCACHE, int RING, bool OVF, int F>
__device__ __forceinline__ DScene shade_scene_lds(const DScene& S0) {
    if constexpr (!NCACHE && JT_KARG_SCENE_LDS) {
        extern __shared__ uint4 dyn_lds[];
        const DScene& K = shade_scene<true>(S0);
        return blob_scene(K, dyn_lds + lds_stack_bytes(OVF, RING, K.stack_need) / 16);
    } else {
        return S0;
    }
}
#define JT_A(f) (karg_reload<F>() ? karg<decltype(DAccum::f)>(offsetof(KArgs, A) + offsetof(DAccum, f)) : A.f)
#define JT_SB (karg_reload<F>() ? karg<int>(offsetof(KArgs, s_begin)) : s_begin)
#define JT_SE (karg_reload<F>() ? karg<int>(offsetof(KArgs, s_end)) : s_end)

// Work units: (8x8 pixel tile t, stream slot q), fetched by whole waves from atomic counters, so
// every wave stays busy until the launch's last units. The tiles are split into 8 bands of rows,
// one per XCD: a wave drains its own XCD's band first (neighbouring pixels share that XCD's L2),
// then helps the other bands. Within a band units are numbered tile-major: a tile's stream slots
// are consecutive units, so the waves running at one time trace the same pixels' samples (the
// first bounces share nodes and texels in the XCD's L2). Measured against stream-major numbering
// (gpurun_out/r05x, two runs each): features2 +4.5 %, ecosys +1.1 %, bathroom1 +0.6 %,
// cornellbox +0.4 %.
constexpr int NBANDS = 8, BAND_STRIDE = 16;

// number of 8x8 tiles a launch covers (DParams tile_stride / tile_offset)
__host__ __device__ __forceinline__ int launch_tiles(const DParams& P) {
    const int all = ((P.width + 7) / 8) * ((P.height + 7) / 8);
    return all > P.tile_offset ? (all - P.tile_offset + P.tile_stride - 1) / P.tile_stride : 0;
}

// ============================================================================ sample streams + per-lane work items
// Sample streams: the samples of a pixel are dealt to k = 2^P.lk streams (local sample t = s -
// first goes to stream t mod k), and each stream keeps its own running mean (src/trace.jl:631-648,
// weight 1/(c + 1) for the stream's c-th sample). A (pixel, stream) item is one lane's work for
// the launch: its samples in order, then one store of the stream's means. Items are independent
// of each other — no item waits for another — so a launch has W·H·min(k, samples) concurrent
// items however few pixels it covers, and the launch ends by combining each pixel's stream means
// in stream order (combine_kernel, weights n_j / n). k = 1 is the reference's own single running
// mean (the image buffer is stream 0): one sample per launch reads and writes it here; a longer
// range runs as chunks of one-sample streams folded in sample order (chain_kernel, jt_trace.hip).
// Results depend on k (fixed per context, jt_get_streams) and not on how a render is split into
// calls or launches.
//
// Per-lane work items: the work units are (8x8 tile, stream), fetched by whole waves, but a lane
// is not tied to its wave's unit: a lane that has finished its item takes the next pixel of its
// wave's current unit at once, and the wave fetches the next unit when every pixel of the
// current one has been handed out. A wave therefore never waits for the slowest lane of a unit;
// lanes hold pixels of at most a few consecutive units, so neighbouring lanes stay spatially
// close. The wave-level hand-out is a ballot and a prefix count (mbcnt): the k-th needy lane
// takes pixel bnext + k.
// JT_ITEM_FIRST_POP: a sample's first node pops run at its start, in the hand-out, where most of
// the wave's lanes start samples together (1: every kernel, 0: none, 2: the binary-order mesh
// kernels only). Measured in round 4 (profiles/r04_ab/knobs*_r04[rs].txt, two runs each), off
// against on: cornellbox +0.4 % (10317/10318 vs 10273/10277 Mrays/s), bathroom1 and ecosys (wide)
// +1.2 % and even, features2 (near, mesh) -1.5 % (2666/2679 vs 2722/2709). 2.
#ifndef JT_ITEM_FIRST_POP
#define JT_ITEM_FIRST_POP 2
#endif
template <bool WIDE, int F>
__host__ __device__ constexpr bool item_first_pop() {
    return JT_ITEM_FIRST_POP == 1 || (JT_ITEM_FIRST_POP == 2 && !WIDE && !ft_none(F));
}
// a lane's item: the pixel's slot tile * 64 + l (l: pixel of the 8x8 tile; jt_create keeps
// tiles below 2^20); ITEM_NONE: no pixel. The item's stream and sample live in the lane's LDS
// slot [11] (its current global sample).
constexpr unsigned ITEM_NONE = 0xffffffffu;

// the image index of an item's pixel (its slot holds the global tile and the pixel of the tile)
__device__ __forceinline__ int item_pixel(unsigned item, const DParams& P, int tiles_x) {
    const int t = (int)(item >> 6), l = (int)(item & 63u);
    return ((t / tiles_x) * 8 + (l >> 3)) * P.width + (t % tiles_x) * 8 + (l & 7);
}
// an item's slot among the launch's tiles (DAccum::part_*): tiles offset, offset + stride, ... are
// launch tiles 0, 1, ...; (t - offset) / stride is exact, and t < 2^20 keeps the float quotient
// within 2^-3 of it. Against the integer division: cornellbox +0.5 %, its 1/8 share +0.9 % (two
// runs each, profiles/r06_ab/slot_float_vs_div_r06d.txt; the division's code raised the kernels'
// spills from 1-2 to 4-6 VGPRs)
__host__ __device__ __forceinline__ int item_slot(unsigned item, const DParams& P) {
    const int t = (int)(item >> 6);
    const int u = (int)((float)(t - P.tile_offset) * (1.0f / (float)P.tile_stride) + 0.5f);
    return u * 64 + (int)(item & 63u);
}
// running-mean weight of global sample s within its stream
__device__ __forceinline__ float stream_weight(const DParams& P, int s) {
    return 1.0f / (float)(((s - P.first) >> P.lk) + 1);
}

#if JT_STAMPS
#define JT_STAMP(x) x
#else
#define JT_STAMP(x)
#endif

template <int SAMPLER, int RING, bool OVF, int COUNT, int F, bool NCACHE, bool WIDE>
__device__ __forceinline__ void trace_body_items(const DScene& S0, const DParams& P0, int s_begin, int s_end,
                                                 const DAccum& A, int* stack) {
    const DScene& S = S0;
    const DParams& P = P0;
    static_assert(lane_lds(F), "the per-lane item body keeps the lane's sample index in LDS");
    const int lane = threadIdx.x & 63;
    const int oslot = (int)blockIdx.x * BLOCK + (int)threadIdx.x;  // the lane's HBM stack-overflow area
    if constexpr ((F & (FT_TEX | FT_ENV)) != 0) {  // the texel-decode LUTs into LDS (tex_lut)
        for (int k = threadIdx.x; k < 512; k += BLOCK) tex_lut[k] = k < 256 ? S.srgb_lut[k] : S.byte_lut[k - 256];
        __syncthreads();
    }
    Counters cnt{0, 0, 0, 0};
    // Paths, scene rays and light queries are counted per wave, never in per-lane registers
    // (three VGPRs live across the traversal loop, spilled and written back every shading
    // phase: 14 GB of scratch write-back per cornellbox launch).
    // WC (mesh kernels): ballots at wave-uniform points, summed in scalar registers (bathroom1
    // +3 %, features2 +1 % over per-lane counters). The FT_NONE kernel, whose light-hit steps run
    // every few iterations, adds to three per-wave LDS words instead (ds_add, no ballot).
    constexpr bool WC = !ft_none(F);
    unsigned w_paths = 0, w_rays = 0, w_lq = 0;
    __shared__ unsigned wave_cnt[WC ? 1 : (BLOCK / 64) * 4];
    unsigned* const wcnt = wave_cnt + (WC ? 0 : (threadIdx.x >> 6) * 4);
    if (!WC && lane < 3) wcnt[lane] = 0u;
    auto lds_count = [&](int k, bool c) {
        if (c) __hip_atomic_fetch_add(wcnt + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    __shared__ float acc_lds[acc_slots(F) * BLOCK];
    float* acc = acc_lds + threadIdx.x;
    int* const acc_i = reinterpret_cast<int*>(acc);
#if JT_STAMPS
    // per-phase wave clocks, step lanes, shading-phase material coherence (scripts/stamps.py)
    unsigned long long t_trav = 0, t_shade = 0, n_trav = 0, n_shade = 0, lanes_p = 0, lanes_n = 0, steps_p = 0, steps_n = 0;
    unsigned long long t_hit = 0, t_fin = 0, t_qb = 0, n_phit = 0, n_fin = 0, idle = 0, n_mph = 0, n_mty = 0, n_mid = 0;
    unsigned long long lanes_sh = 0, lanes_hit = 0, t_start = 0, n_start = 0, lanes_start = 0;
#endif
    const int tiles_x = (P.width + 7) / 8, tiles = launch_tiles(P);
    const int kstr = 1 << P.lk;
    // stream slots of this launch: q = 0 .. nq-1 starts at global sample s_begin + q
    const int nq = s_end - s_begin < kstr ? s_end - s_begin : kstr;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    int band_k = 0;
    int ut = 0, uq = 0, bnext = 64;  // the wave's current unit (tile, stream slot) and its next pixel to hand out
    bool drained = false;            // every band's units handed out
    unsigned item = ITEM_NONE;       // the lane's pixel (ITEM_* above)
    bool next_sample = false;        // the lane's next sample starts at the top of the iteration
    Aov aov{acc, 0.0f, P.first, P.lk};
    Path st;
    st.pk = acc + acc_base_slots(F) * BLOCK;
    Trav T;
    T.sp = -1;
    T.nprim = 0;
    T.nxt = W_EMPTY;
    for (;;) {
        JT_STAMP(const unsigned long long ts0 = __builtin_amdgcn_s_memtime());
        // ---- hand out pixels to the lanes without one (wave-uniform control); a lane taking an
        // item starts from its stream's means so far (zero for the stream's first sample)
        bool start = next_sample;
        for (;;) {
            const unsigned long long needm = __builtin_amdgcn_ballot_w64(item == ITEM_NONE);
            if (!needm || drained) break;
            if (bnext >= 64) {  // the next unit of this XCD's band, or of the next band
                const int band = (int)((xcc + (unsigned)band_k) & (NBANDS - 1));
                // JT_BAND_STRIP > 1: bands of whole tile rows, each walked in strips of that many
                // rows, column by column, so the tiles in flight on an XCD form a compact block
                // (their rays share nodes and texels in L2).
                // A tile share (tile_stride D) whose D divides the tile columns is a grid of
                // tiles_x / D columns in launch-tile numbering and is walked the same way.
                constexpr int STRIP = JT_BAND_STRIP;
                const int gx = tiles_x % P.tile_stride == 0 ? tiles_x / P.tile_stride : 0;
                const bool strips = STRIP > 1 && gx > 0;
                const int tiles_y = (P.height + 7) / 8;
                const int bt0 = strips ? band * tiles_y / NBANDS * gx : band * tiles / NBANDS;
                const int bn = strips ? (band + 1) * tiles_y / NBANDS * gx - bt0 : (band + 1) * tiles / NBANDS - bt0;
                unsigned unit = 0;
                if (lane == 0) unit = atomicAdd(JT_A(work) + band * BAND_STRIDE, 1u);
                unit = __builtin_amdgcn_readfirstlane(unit);
                if (unit >= (unsigned)bn * (unsigned)nq) {
                    if (++band_k >= NBANDS) drained = true;
                    continue;
                }
                uq = (int)(unit % (unsigned)nq);  // tile-major (NBANDS above)
                const int tu = (int)(unit / (unsigned)nq);
                int tile = bt0 + tu;
                if (strips) {
                    const int rows = bn / gx, sidx = tu / (STRIP * gx);
                    const int v = tu - sidx * STRIP * gx, h = rows - sidx * STRIP < STRIP ? rows - sidx * STRIP : STRIP;
                    tile = bt0 + (sidx * STRIP + v % h) * gx + v / h;
                }
                ut = tile * P.tile_stride + P.tile_offset;
                bnext = 0;
            }
            const int nneed = lane_count(needm), take = nneed < 64 - bnext ? nneed : 64 - bnext;
            const int rank = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(needm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)needm, 0u));
            if (item == ITEM_NONE && rank < take) {
                const int l = bnext + rank;
                const int i = (ut % tiles_x) * 8 + (l & 7), j = (ut / tiles_x) * 8 + (l >> 3);
                // a pixel outside the image (edge tiles) is skipped: the lane takes another
                if (i < P.width && j < P.height) {
                    item = (unsigned)(ut * 64 + l);
                    start = true;
                    const int s = JT_SB + uq;
                    acc_i[11 * BLOCK] = s;
                    const int pixel = j * P.width + i;
                    float4 im = make_float4(0, 0, 0, 0), al = im, nr = im;
                    int h = 0;
                    if (s - P.first >= kstr) {  // the stream has earlier samples (an earlier launch)
                        if (P.lk == 0) {
                            im = JT_A(image)[pixel];
                            al = JT_A(albedo)[pixel];
                            nr = JT_A(normal)[pixel];
                            h = (int)JT_A(hits)[pixel];
                        } else {
                            const size_t o = (size_t)((s - P.first) & (kstr - 1)) * (size_t)JT_A(nslot) +
                                             (size_t)item_slot(item, P);
                            im = JT_A(part_img)[o];
                            al = JT_A(part_alb)[o];
                            nr = JT_A(part_nrm)[o];
                            h = __float_as_int(al.w);
                        }
                    }
                    acc[0] = im.x;
                    acc[BLOCK] = im.y;
                    acc[2 * BLOCK] = im.z;
                    acc[3 * BLOCK] = im.w;
                    acc[4 * BLOCK] = al.x;
                    acc[5 * BLOCK] = al.y;
                    acc[6 * BLOCK] = al.z;
                    acc[7 * BLOCK] = nr.x;
                    acc[8 * BLOCK] = nr.y;
                    acc[9 * BLOCK] = nr.z;
                    acc_i[10 * BLOCK] = h;
                }
            }
            bnext += take;
        }
        // ---- every lane starting a sample (a new item, or the next sample of its stream): the
        // camera ray (trace_sample's prologue) and its query's first pops, where many lanes share them
        next_sample = false;
        if (start) {
            const int sample = acc_i[11 * BLOCK];
            const int pixel = item_pixel(item, P, tiles_x);
            if (!ft_none(F)) acc[12 * BLOCK] = stream_weight(P, sample);
            const DParams& P = karg_params<karg_params_on<SAMPLER, F>()>(P0);
            start_path<F>(P, pixel % P.width, pixel / P.width, pixel, sample, st);
            query_start<WIDE>(S, T, st.o, st.d, -1, stack);
            if (!WC) lds_count(1, true);
            if constexpr (item_first_pop<WIDE, F>()) {
#pragma unroll
                for (int k = 0; k < (!ft_none(F) && (F & FT_LINL) ? JT_FIRST_POP : JT_FIRST_POP_NONE); k++)
                    if (wants_node<WIDE>(T)) node_step_any<WIDE, RING, OVF, COUNT, NCACHE, F>(S, T, stack, oslot, cnt);
            }
        }
        if (WC) w_rays += lane_count(__builtin_amdgcn_ballot_w64(start));
#if JT_STAMPS
        const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
        t_start += ts1 - ts0;
        n_start++;
        lanes_start += lane_count(__builtin_amdgcn_ballot_w64(start));
#endif
        if (__builtin_amdgcn_ballot_w64(item != ITEM_NONE) == 0) break;  // drained, and every lane is done
        // ---- traversal phase: step every lane with a query in flight until enough lanes wait.
        // Each iteration runs ONE step kind — primitive tests or stack pops — picked by a biased
        // lane vote (a wave-uniform branch), so the SIMD executes one code path per iteration; a
        // lane's own sequence of steps is unchanged, it only waits while the other kind runs.
        // Light-hit steps (path sampler, matte scenes whose light chains cannot run inline): a
        // lane whose sample_lights_pdf query has finished does not wait for the shading phase.
        constexpr bool LSTEP = light_steps(SAMPLER, F);
        for (;;) {
            const bool wantp = T.nprim > 0;
            const bool wantn = wants_node<WIDE>(T);
            const bool waiting = query_done<WIDE>(T);
            const int np = lane_count(__builtin_amdgcn_ballot_w64(wantp));
            const int nn = lane_count(__builtin_amdgcn_ballot_w64(wantn));
            int nw = lane_count(__builtin_amdgcn_ballot_w64(waiting));
            const int nb = np + nn;
            if (LSTEP && !S.light_inline) {
                const bool wantl = waiting && st.phase == PH_LIGHT;
                const int nl = lane_count(__builtin_amdgcn_ballot_w64(wantl));
                if (nl > 0 && (nl >= P.light_lanes || nb == 0)) {
                    bool c_lq = false, c_ray = false;
                    if (wantl && rerun_tie<WIDE>(S, T, st.o, st.d, S.lights[st.li].instance, stack)) {
                        // an exact-t tie: the query runs again in the reference's order
                    } else if (wantl) {
                        if (light_hit<F>(S, P, st, query_hit(T))) {
                            st.phase = PH_FINISH;
                        } else if (st.phase == PH_LIGHT) {
                            if (WC) c_lq = true;
                            else lds_count(2, true);
                            query_start<WIDE>(S, T, st.o, st.d, S.lights[st.li].instance, stack);
                        } else {
                            if (WC) c_ray = true;
                            else lds_count(1, true);
                            query_start<WIDE>(S, T, st.o, st.d, -1, stack);
                        }
                    }
                    if (WC) {
                        w_lq += lane_count(__builtin_amdgcn_ballot_w64(c_lq));
                        w_rays += lane_count(__builtin_amdgcn_ballot_w64(c_ray));
                    }
                    continue;
                }
                nw -= nl;
            }
            if (nb == 0 || nw >= (nb + nw < P.wait_lanes ? nb + nw : P.wait_lanes)) break;
#if JT_STAMPS
            n_trav++;
            idle += 64 - lane_count(__builtin_amdgcn_ballot_w64(item != ITEM_NONE));
            if (np * JT_VOTE_P >= nn * JT_VOTE_N) { steps_p++; lanes_p += np; } else { steps_n++; lanes_n += nn; }
#endif
            if (JT_RAY_FROM_PATH && !(F & FT_XFORM)) {
                // without instance transforms a query's ray is its path's (st.o, st.d), unchanged
                // while the query runs: re-reading it here keeps one copy, not two, live across
                // the loop (register renaming only, no instructions)
                T.lo = st.o;
                T.ld = st.d;
            }
            if (np * JT_VOTE_P >= nn * JT_VOTE_N) {
                if (T.nprim > 0) prim_step<COUNT, F>(S, T, cnt);
            } else {
                // JT_NODE_REPEAT pops per node iteration: a lane whose next step is again a
                // stack pop takes it at once (the same steps in the same per-lane order, less
                // per-iteration vote and loop overhead)
                constexpr int NREP = ft_none(F) ? JT_NODE_REPEAT_NONE : JT_NODE_REPEAT;
#pragma unroll
                for (int k = 0; k < NREP; k++)
                    if (wants_node<WIDE>(T)) node_step_any<WIDE, RING, OVF, COUNT, NCACHE, F>(S, T, stack, oslot, cnt);
            }
        }
#if JT_STAMPS
        const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
        t_trav += ts2 - ts1;
        n_shade++;
        lanes_sh += lane_count(__builtin_amdgcn_ballot_w64(query_done<WIDE>(T)));
        {
            int mid = -1, mt = -1;
            if (query_done<WIDE>(T) && st.phase == PH_SCENE && T.h_inst >= 0) {
                mid = S.inst_shade[T.h_inst].material;
                mt = (F & FT_MAT) ? S.materials[mid].type : (int)M_MATTE;
            }
            if (__builtin_amdgcn_ballot_w64(mt >= 0)) {
                n_mph++;
                lanes_hit += lane_count(__builtin_amdgcn_ballot_w64(mt >= 0));
                for (int ty = 0; ty <= (int)M_GLTFPBR; ty++) n_mty += __builtin_amdgcn_ballot_w64(mt == ty) ? 1u : 0u;
                bool counted = mt < 0;
                for (;;) {
                    const unsigned long long m = __builtin_amdgcn_ballot_w64(!counted);
                    if (!m) break;
                    const int v = __shfl(mid, __ffsll((long long)m) - 1);
                    counted = counted || mid == v;
                    n_mid++;
                }
            }
        }
        unsigned long long ts3 = ts2, ts4 = ts2;
#endif
        // ---- shading phase: every waiting lane consumes its hit and issues its next query; a
        // near-first query that saw an exact-t tie first runs again in the reference's order
        constexpr bool LINL = (F & (FT_LINL | FT_NOIL)) != 0;
        {
            const bool tie = query_done<WIDE>(T) && (T.nh & (TIE_SEEN | REF_RERUN)) == TIE_SEEN &&
                             !(LSTEP && st.phase == PH_FINISH);
            if (S.order_flip && __builtin_amdgcn_ballot_w64(tie))
                if (tie) rerun_tie<WIDE>(S, T, st.o, st.d, SAMPLER == 1 && !LINL && st.phase == PH_LIGHT ? S.lights[st.li].instance : -1, stack);
        }
        bool c_path = false, c_lq = false, c_ray = false;
        unsigned n_inl = 0;
        if (query_done<WIDE>(T)) {
            const DParams& P = karg_params<karg_params_on<SAMPLER, F>()>(P0);
            const DScene SL = shade_scene_lds<NCACHE, RING, OVF, F>(S0);
            const DScene& S = NCACHE ? shade_scene<karg_scene<NCACHE, F>()>(S0) : SL;
            bool alive = true;
            // no light query ever leaves the shading phase (FT_LINL), or none exists (FT_NOIL)
            const bool light = SAMPLER == 1 && !LINL && st.phase == PH_LIGHT;
            bool done;
            if (LSTEP && st.phase == PH_FINISH) done = true;
            else if (light) done = light_hit<F>(S, P, st, query_hit(T));
            else if (SAMPLER == 2) done = naive_hit<F>(S, P, st, query_hit(T), aov, cnt.shades);
            else done = path_hit<F>(S, P, st, query_hit(T), aov, cnt.shades);
            if (SAMPLER == 1 && !done && st.phase == PH_LIGHT && chains_inline(F, S)) {
                unsigned nlq = 0;
                done = light_chain<WIDE, RING, OVF, COUNT, NCACHE, F>(S, P, st, T, stack, oslot, cnt, [&] {
                    if (WC) nlq++;
                    else lds_count(2, true);
                });
                if (WC) n_inl += nlq;
            }
#if JT_STAMPS
            ts3 = __builtin_amdgcn_s_memtime();
            n_phit++;
#endif
            if (done) {
                // trace_sample epilogue (src/trace.jl:625-648), into the item's stream mean
                if (WC) c_path = true;
                else lds_count(0, true);
                v3 radiance = st.radiance<F>();
                if (!all_finite(radiance)) radiance = V3(0, 0, 0);
                const float mr = max3(radiance);
                if (mr > P.clamp) radiance = radiance * (P.clamp / mr);
                const float w = aov.w<F>();
                const float omw = 1 - w;
                const bool hit = st.flag(F_HIT);
                const bool env = !hit && !P.envhidden && S.nenvs != 0;
                const v4 target = (hit || env) ? V4(radiance.x, radiance.y, radiance.z, 1) : V4(0, 0, 0, 0);
                // no bounce-0 surface was accepted: st.d is still the camera ray direction
                if (!hit) aov_update<F>(aov, env ? V3(1, 1, 1) : V3(0, 0, 0), -st.d);
                acc[0] = acc[0] * omw + target.x * w;
                acc[BLOCK] = acc[BLOCK] * omw + target.y * w;
                acc[2 * BLOCK] = acc[2 * BLOCK] * omw + target.z * w;
                acc[3 * BLOCK] = acc[3 * BLOCK] * omw + target.w * w;
                if (hit || env) acc_i[10 * BLOCK] += 1;
                alive = false;
                T.sp = -1;
                const int sample = acc_i[11 * BLOCK];
                if (sample + kstr >= JT_SE) {
                    // the item is complete: store its stream's means (plain stores: no other item
                    // of this launch reads them; the combine kernel runs after the launch)
                    const int pixel = item_pixel(item, P, tiles_x);
                    const float4 im = make_float4(acc[0], acc[BLOCK], acc[2 * BLOCK], acc[3 * BLOCK]);
                    if (P.lk == 0) {
                        JT_A(image)[pixel] = im;
                        JT_A(albedo)[pixel] = make_float4(acc[4 * BLOCK], acc[5 * BLOCK], acc[6 * BLOCK], 0.0f);
                        JT_A(normal)[pixel] = make_float4(acc[7 * BLOCK], acc[8 * BLOCK], acc[9 * BLOCK], 0.0f);
                        JT_A(hits)[pixel] = (long long)acc_i[10 * BLOCK];
                    } else {
                        const size_t o = (size_t)((sample - P.first) & (kstr - 1)) * (size_t)JT_A(nslot) +
                                         (size_t)item_slot(item, P);
                        JT_A(part_img)[o] = im;
                        JT_A(part_alb)[o] = make_float4(acc[4 * BLOCK], acc[5 * BLOCK], acc[6 * BLOCK], __int_as_float(acc_i[10 * BLOCK]));
                        JT_A(part_nrm)[o] = make_float4(acc[7 * BLOCK], acc[8 * BLOCK], acc[9 * BLOCK], 0.0f);
                    }
                    item = ITEM_NONE;
                } else {
                    acc_i[11 * BLOCK] = sample + kstr;  // started at the top of the next iteration
                    next_sample = true;
                }
            }
#if JT_STAMPS
            ts4 = __builtin_amdgcn_s_memtime();
            if (__builtin_amdgcn_ballot_w64(done)) n_fin++;
#endif
            if (alive) {
                if (SAMPLER == 1 && !LINL && st.phase == PH_LIGHT) {
                    if (WC) c_lq = true;
                    else lds_count(2, true);
                    query_start<WIDE>(S, T, st.o, st.d, S.lights[st.li].instance, stack);
                } else {
                    if (WC) c_ray = true;
                    else lds_count(1, true);
                    query_start<WIDE>(S, T, st.o, st.d, -1, stack);
                }
                // the query's first pop (TLAS root, or the light instance and its BLAS root) here,
                // where most of the wave's lanes take part, rather than in a sparser traversal step
#pragma unroll
                for (int k = 0; k < (!ft_none(F) && (F & FT_LINL) ? JT_FIRST_POP : JT_FIRST_POP_NONE); k++)
                    if (wants_node<WIDE>(T)) node_step_any<WIDE, RING, OVF, COUNT, NCACHE, F>(S, T, stack, oslot, cnt);
            }
        }
#if JT_STAMPS
        const unsigned long long ts5 = __builtin_amdgcn_s_memtime();
        t_shade += ts5 - ts2;
        t_hit += ts3 - ts2;
        t_fin += ts4 - ts3;
        t_qb += ts5 - ts4;
#endif
        if (WC) {
            w_paths += lane_count(__builtin_amdgcn_ballot_w64(c_path));
            w_lq += lane_count(__builtin_amdgcn_ballot_w64(c_lq));
            w_rays += lane_count(__builtin_amdgcn_ballot_w64(c_ray));
            if (SAMPLER == 1 && chains_inline(F, S)) w_lq += __builtin_amdgcn_readfirstlane(wave_sum(n_inl));
        }
    }
#if JT_STAMPS
    if (lane == 0) {
        unsigned long long* dbg = A.counters + 8;
        const unsigned long long v[24] = {t_trav, t_shade, n_trav,  n_shade, lanes_p, lanes_n,  steps_p, steps_n,
                                          0,      t_hit,   t_fin,   t_qb,    0,       n_phit,   n_fin,   idle,
                                          n_mph,  n_mty,   n_mid,   lanes_sh, lanes_hit, t_start, n_start, lanes_start};
        for (int k = 0; k < 24; k++) atomicAdd(dbg + k, v[k]);
    }
#endif
    // one atomic per counter per wave (the wave's own LDS adds precede this read in program order)
    const unsigned wv[3] = {w_paths, w_rays, w_lq};
    unsigned v[7] = {0u, 0u, 0u, cnt.nodes, cnt.instances, cnt.prims, COUNT ? cnt.shades : 0u};
#pragma unroll
    for (int k = 0; k < 7; k++) {
        unsigned sum = k < 3 ? (WC ? wv[k] : wcnt[k]) : wave_sum(v[k]);
        if (lane == 0 && sum) atomicAdd(&A.counters[k], (unsigned long long)sum);
    }
}

// The launch's last step when k > 1 (combine_kernel, jt_trace.hip): each pixel's stream means
// combined in stream order, mean = sum_j mean_j * w_j over the streams with samples (w_j = n_j /
// n, host-computed in double and rounded once), hits = sum_j hits_j.
struct DCombine {
    float w[JT_MAX_STREAMS];
    int ns;  // streams with samples: min(k, n)
};
// Occupancy request (waves per SIMD); JT_WAVES=0 leaves it to the compiler. The LDS-mode
// FT_NONE kernel (cornellbox: 96 VGPRs, LDS for 5 workgroups per CU with the stack sized to the
// scene) asks for JT_WAVES_NONE: measured +4 % over 4 waves with its wait_lanes of 56.
#ifndef JT_WAVES
#define JT_WAVES 0
#endif
#ifndef JT_WAVES_NONE
#define JT_WAVES_NONE 5
#endif
#if JT_WAVES > 0
#define JT_WAVES_PER_EU __attribute__((amdgpu_waves_per_eu(JT_WAVES, JT_WAVES)))
#define JT_WAVES_PER_EU_F(F) \
    __attribute__((amdgpu_waves_per_eu(ft_none(F) ? JT_WAVES_NONE : JT_WAVES, ft_none(F) ? JT_WAVES_NONE : JT_WAVES)))
#else
#define JT_WAVES_PER_EU
#define JT_WAVES_PER_EU_F(F)
#endif
// LDS-mode stack bytes per workgroup: a RING-entry ring with HBM overflow, else the scene's bound
__host__ __device__ constexpr size_t lds_stack_bytes(bool ovf, int ring, int need) {
    return (size_t)(ovf ? ring : need) * BLOCK * 4;
}

// the scene arrays of the LDS blob (small-scene mode; offsets from jt_create)
__device__ __forceinline__ DScene blob_scene(const DScene& S, const uint4* blob) {
    DScene L = S;
    L.nodes = reinterpret_cast<const DNode*>(blob + S.o_nodes);
    L.wnodes = reinterpret_cast<const DWide*>(blob + S.o_wnodes);
    L.prims = reinterpret_cast<const float4*>(blob + S.o_prims);
    L.inst_trav = reinterpret_cast<const DInstTrav*>(blob + S.o_inst_trav);
    L.inst_blas = reinterpret_cast<const int4*>(blob + S.o_inst_blas);
    L.inst_shade = reinterpret_cast<const DInstShade*>(blob + S.o_inst_shade);
    L.shapes = reinterpret_cast<const DShape*>(blob + S.o_shapes);
    L.pos = reinterpret_cast<const float4*>(blob + S.o_pos);
    L.nrm = reinterpret_cast<const float4*>(blob + S.o_nrm);
    L.tc = reinterpret_cast<const float2*>(blob + S.o_tc);
    L.col = reinterpret_cast<const float4*>(blob + S.o_col);
    L.elems = reinterpret_cast<const int4*>(blob + S.o_elems);
    L.enrm = reinterpret_cast<const float4*>(blob + S.o_enrm);
    L.enrm_id = reinterpret_cast<const float4*>(blob + S.o_enrm_id);
    L.materials = reinterpret_cast<const DMaterial*>(blob + S.o_materials);
    L.lights = reinterpret_cast<const DLight*>(blob + S.o_lights);
    L.light_hit = reinterpret_cast<const int4*>(blob + S.o_light_hit);
    L.light_elems = reinterpret_cast<const float4*>(blob + S.o_light_elems);
    L.cdf = reinterpret_cast<const float*>(blob + S.o_cdf);
    return L;
}

// HBM mode: the scene is read from global memory (L2/MALL-resident); stack in static LDS.
template <int SAMPLER, int RING, bool OVF, int COUNT, int F, bool WIDE>
__global__ __launch_bounds__(BLOCK) JT_WAVES_PER_EU void trace_kernel(DScene S, DParams P, int s_begin, int s_end, DAccum A) {
    __shared__ int lds_stack[RING * BLOCK];
    trace_body_items<SAMPLER, RING, OVF, COUNT, F, true, WIDE>(S, P, s_begin, s_end, A, lds_stack + threadIdx.x);
}

// LDS mode (small scenes): the workgroup stages the scene blob into LDS once; every node,
// instance, primitive and shading record is then a ds_read instead of a vector-memory load
// through the TA/TD path (the measured limiter of the HBM-mode kernel).
template <int SAMPLER, int RING, bool OVF, int COUNT, int F, bool WIDE>
__global__ __launch_bounds__(BLOCK) JT_WAVES_PER_EU_F(F) void trace_kernel_lds(DScene S, DParams P, int s_begin, int s_end, DAccum A) {
    extern __shared__ uint4 dyn_lds[];
    // the stack takes the first bytes (lds_stack_bytes), the blob follows
    uint4* blob = dyn_lds + lds_stack_bytes(OVF, RING, S.stack_need) / 16;
    for (int k = threadIdx.x; k < S.blob_n16; k += BLOCK) blob[k] = S.blob[k];
    __syncthreads();
    const DScene L = blob_scene(S, blob);
    trace_body_items<SAMPLER, RING, OVF, COUNT, F, false, WIDE>(L, P, s_begin, s_end, A, reinterpret_cast<int*>(dyn_lds) + threadIdx.x);
}

// Persistent launch: as many workgroups as the device holds at once (capped by the number of
// tiles), each wave then pulls work units until the launch's units are exhausted.
// LDSK: the specialisation also has an LDS-mode kernel (the large-scene masks run in HBM mode).
template <int SAMPLER, int RING, bool OVF, int COUNT, int F, bool LDSK, bool WIDE>
hipError_t launch_t(const DScene& S, const DParams& P, int s0, int s1, const DAccum& A, hipStream_t st, int cus) {
    // one wave per work unit (tile, stream slot) at most
    const long long units = (long long)launch_tiles(P) * std::min(s1 - s0, 1 << P.lk);
    const int want = (int)std::min<long long>((units + BLOCK / 64 - 1) / (BLOCK / 64), 1 << 30);
    if (want == 0) return hipSuccess;  // a multi-device share without tiles (tiny image)
    int per_cu = 0;
    hipError_t e;
    if constexpr (LDSK) {
        if (S.blob_n16 > 0) {
        const size_t lds = lds_stack_bytes(OVF, RING, S.stack_need) + (size_t)S.blob_n16 * 16;
        const void* k = (const void*)trace_kernel_lds<SAMPLER, RING, OVF, COUNT, F, WIDE>;
        if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)) != hipSuccess) return e;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, BLOCK, lds) != hipSuccess || per_cu < 1) per_cu = 1;
        const int nwg = std::min(want, std::min(per_cu, 8) * cus);  // <= 8 per CU: the overflow area's bound
        hipLaunchKernelGGL((trace_kernel_lds<SAMPLER, RING, OVF, COUNT, F, WIDE>), dim3(nwg), dim3(BLOCK), lds, st, S, P, s0, s1, A);
        return hipGetLastError();
        }
    }
    const void* k = (const void*)trace_kernel<SAMPLER, RING, OVF, COUNT, F, WIDE>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, BLOCK, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    const int nwg = std::min(want, std::min(per_cu, 8) * cus);
    hipLaunchKernelGGL((trace_kernel<SAMPLER, RING, OVF, COUNT, F, WIDE>), dim3(nwg), dim3(BLOCK), 0, st, S, P, s0, s1, A);
    return hipGetLastError();
}

// Feature specialisations compiled per stack configuration (besides FT_ALL): FT_NONE for small
// scenes with a 16-entry stack (cornellbox), and three masks for large HBM-mode scenes with the
// ring + HBM overflow stack — textured, attributed meshes (bathroom1), plus environments
// (ecosys), plus quads (features2). FT_NONE, FT_MESH and FT_MESH_ENV_QUAD are FT_LINL builds
// (light chains inline, no light-hit steps); a second FT_NONE build keeps the light-hit steps.
constexpr int FT_MESH = FT_TEX | FT_ATTR | FT_MAT | FT_OPAC | FT_XFORM;
constexpr int FT_MESH_ENV = FT_MESH | FT_ENV;
constexpr int FT_MESH_ENV_QUAD = FT_MESH_ENV | FT_QUAD;
// the kernel mask a scene with feature bits `feat` runs with: the smallest compiled superset.
// `linl`: the scene's light chains can run inline (DScene::light_inline), which the FT_LINL
// builds need; FT_MESH_ENV is built for scenes without instance lights (FT_NOIL: no light
// queries at all; the chain code cost ecosys 4 spilled VGPRs). Matte scenes
// whose chains cannot run inline get the FT_NONE build with light-hit steps.
inline int kernel_mask(int feat, int need, int ring, bool lds, bool linl, bool inst_light) {
    if (need <= 16) return feat == FT_NONE ? (linl ? FT_NONE | FT_LINL : FT_NONE) : FT_ALL;
    if (ring > 16 || lds) return FT_ALL;
    for (int m : {FT_MESH | FT_LINL, FT_MESH_ENV | FT_NOIL, FT_MESH_ENV_QUAD | FT_LINL})
        if (!(feat & ~m & ~(FT_LINL | FT_NOIL)) && ((m & FT_LINL) ? linl : !inst_light)) return m;
    return FT_ALL;
}

// Kernel configurations: (stack ring, HBM overflow, feature mask, LDS-mode kernel too), each in
// the binary traversal (ID 0-7) and the wide one (ID + 8, JT_TRAVERSAL_WIDE). Each is compiled
// in its own translation unit (jt_kv.hip with JT_VARIANT = its index) for both samplers and both
// counter levels; launch_s (jt_trace.hip) dispatches among them.
constexpr int NUM_BASE_CONFIGS = 8;
template <int ID>
struct LaunchConfig;
#define JT_LAUNCH_CONFIG(ID, R, O, F, L)                            \
    template <>                                                      \
    struct LaunchConfig<ID> {                                        \
        static constexpr int ring = R;                               \
        static constexpr bool ovf = O;                               \
        static constexpr int feat = F;                               \
        static constexpr bool lds = L;                               \
        static constexpr bool wide = false;                          \
    };                                                               \
    template <>                                                      \
    struct LaunchConfig<ID + NUM_BASE_CONFIGS> : LaunchConfig<ID> {  \
        static constexpr bool wide = true;                           \
    };
JT_LAUNCH_CONFIG(0, 16, false, FT_NONE | FT_LINL, true)  // small scenes, matte triangles (cornellbox)
JT_LAUNCH_CONFIG(1, 16, false, FT_ALL, true)             // small scenes, any features
JT_LAUNCH_CONFIG(2, 16, true, FT_MESH | FT_LINL, false)  // deep BVHs: textured meshes (bathroom1)
JT_LAUNCH_CONFIG(3, 16, true, FT_MESH_ENV | FT_NOIL, false)  // + environments, no instance lights (ecosys)
JT_LAUNCH_CONFIG(4, 16, true, FT_MESH_ENV_QUAD | FT_LINL, false)  // + quads (features2)
JT_LAUNCH_CONFIG(5, 16, true, FT_ALL, true)              // deep BVHs, any features
JT_LAUNCH_CONFIG(6, 32, true, FT_ALL, true)              // a 32-entry LDS ring (JT_LDS_STACK)
JT_LAUNCH_CONFIG(7, 16, false, FT_NONE, true)            // matte triangles, light chains through the traversal
#undef JT_LAUNCH_CONFIG
constexpr int NUM_LAUNCH_CONFIGS = 2 * NUM_BASE_CONFIGS;

template <int ID, int SAMPLER, int COUNT>
hipError_t launch_cfg(const DScene& S, const DParams& P, int s0, int s1, const DAccum& A, hipStream_t st, int cus) {
    using C = LaunchConfig<ID>;
    return launch_t<SAMPLER, C::ring, C::ovf, COUNT, C::feat, C::lds, C::wide>(S, P, s0, s1, A, st, cus);
}
// explicit instantiation (JT_KV_INSTANTIATE, in jt_kv.hip) or declaration (elsewhere) of one
// configuration for both samplers and both counter levels
#define JT_KV_FOR(ID, KW)                                                                                    \
    KW hipError_t launch_cfg<ID, 1, 0>(const DScene&, const DParams&, int, int, const DAccum&, hipStream_t, int); \
    KW hipError_t launch_cfg<ID, 1, 1>(const DScene&, const DParams&, int, int, const DAccum&, hipStream_t, int); \
    KW hipError_t launch_cfg<ID, 2, 0>(const DScene&, const DParams&, int, int, const DAccum&, hipStream_t, int); \
    KW hipError_t launch_cfg<ID, 2, 1>(const DScene&, const DParams&, int, int, const DAccum&, hipStream_t, int);

}  // namespace jtk
