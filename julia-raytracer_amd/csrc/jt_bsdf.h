// jt_bsdf.h — BSDF lobes and the lobe dispatch, per lane (src/shading.jl, src/trace.jl:692-966,
// 1086-1115). Operation order follows the reference expressions; see jt_device.h for the
// float contract.
#pragma once

#include "jt_device.h"

namespace jtd {

enum { M_MATTE = 0, M_GLOSSY, M_REFLECTIVE, M_TRANSPARENT, M_REFRACTIVE, M_SUBSURFACE, M_VOLUMETRIC, M_GLTFPBR };

// MaterialPoint (src/scene.jl:266-320)
struct MatPoint {
    int type;
    v3 emission, color;
    float opacity, roughness, metallic, ior;
    v3 density, scattering;
    float scanisotropy, trdepth;
};

__device__ __forceinline__ v3 up_normal(v3 normal, v3 outgoing) { return dot(normal, outgoing) <= 0 ? -normal : normal; }

// fresnel_dielectric (src/shading.jl:695-714)
__device__ __forceinline__ float fresnel_dielectric(float eta, v3 normal, v3 outgoing) {
    float cosw = __builtin_fabsf(dot(normal, outgoing));
    float sin2 = 1 - cosw * cosw;
    float eta2 = eta * eta;
    float cos2t = 1 - sin2 / eta2;
    if (cos2t < 0) return 1;
    float t0 = __builtin_sqrtf(cos2t);
    float t1 = eta * t0;
    float t2 = eta * cosw;
    float rs = (cosw - t1) / (cosw + t1);
    float rp = (t0 - t2) / (t0 + t2);
    return (rs * rs + rp * rp) / 2;
}
// fresnel_conductor (src/shading.jl:831-851) with etak = 0 (the only use in the hot path)
__device__ __forceinline__ float fresnel_conductor1(float eta, float etak, float cosw, float cos2, float sin2) {
    float eta2 = eta * eta, etak2 = etak * etak;
    float t0 = (eta2 - etak2) - sin2;
    float a2plusb2 = __builtin_sqrtf(t0 * t0 + (4 * eta2) * etak2);
    float t1 = a2plusb2 + cos2;
    float a = __builtin_sqrtf((a2plusb2 + t0) / 2);
    float t2 = (2 * a) * cosw;
    float rs = (t1 - t2) / (t1 + t2);
    float t3 = cos2 * a2plusb2 + sin2 * sin2;
    float t4 = t2 * sin2;
    float rp = rs * (t3 - t4) / (t3 + t4);
    return (rp + rs) / 2;
}
__device__ __forceinline__ v3 fresnel_conductor(v3 eta, v3 normal, v3 outgoing) {
    float cosw = dot(normal, outgoing);
    if (cosw <= 0) return V3(0, 0, 0);
    cosw = jl_clamp(cosw, -1.0f, 1.0f);
    float cos2 = cosw * cosw;
    float sin2 = jl_clamp(1 - cos2, 0.0f, 1.0f);
    return V3(fresnel_conductor1(eta.x, 0.0f, cosw, cos2, sin2), fresnel_conductor1(eta.y, 0.0f, cosw, cos2, sin2),
              fresnel_conductor1(eta.z, 0.0f, cosw, cos2, sin2));
}
__device__ __forceinline__ v3 reflectivity_to_eta(v3 r) {  // src/shading.jl:820-823
    float a = __builtin_sqrtf(jl_clamp(r.x, 0.0f, 0.99f));
    float b = __builtin_sqrtf(jl_clamp(r.y, 0.0f, 0.99f));
    float c = __builtin_sqrtf(jl_clamp(r.z, 0.0f, 0.99f));
    return V3((1 + a) / (1 - a), (1 + b) / (1 - b), (1 + c) / (1 - c));
}
// basis_fromz (src/shading.jl:724-732)
__device__ __forceinline__ m3 basis_fromz(v3 v) {
    v3 z = normalize(v);
    float sign = __builtin_copysignf(1.0f, z.z);
    float a = -1.0f / (sign + z.z);
    float b = z.x * z.y * a;
    return m3{V3(1.0f + sign * z.x * z.x * a, sign * b, -sign * z.x), V3(b, sign + z.y * z.y * a, -z.y), z};
}
// sample_hemisphere_cos (src/shading.jl:716-722)
__device__ __forceinline__ v3 sample_hemisphere_cos(v3 normal, v2 ruv) {
    float z = __builtin_sqrtf(ruv.y);
    float r = __builtin_sqrtf(1 - z * z);
    float phi = 2 * pif * ruv.x;
    float s, c;
    jl_sincos(phi, &s, &c);
    v3 local = V3(r * c, r * s, z);
    return normalize(mul(basis_fromz(normal), local));
}
// GGX microfacet_distribution / shadowing / sampling (src/shading.jl:734-816)
__device__ __forceinline__ float microfacet_distribution(float roughness, v3 normal, v3 halfway) {
    float cosine = dot(normal, halfway);
    if (cosine <= 0) return 0;
    float r2 = roughness * roughness;
    float c2 = cosine * cosine;
    return r2 / (pif * (c2 * r2 + 1 - c2) * (c2 * r2 + 1 - c2));
}
__device__ __forceinline__ float microfacet_shadowing1(float roughness, v3 normal, v3 halfway, v3 direction) {
    float cosine = dot(normal, direction);
    float cosineh = dot(halfway, direction);
    if (cosine * cosineh <= 0) return 0;
    float r2 = roughness * roughness;
    float c2 = cosine * cosine;
    return 2 * __builtin_fabsf(cosine) / (__builtin_fabsf(cosine) + __builtin_sqrtf(c2 - r2 * c2 + r2));
}
__device__ __forceinline__ float microfacet_shadowing(float roughness, v3 normal, v3 halfway, v3 outgoing,
                                                      v3 incoming) {
    return microfacet_shadowing1(roughness, normal, halfway, outgoing) *
           microfacet_shadowing1(roughness, normal, halfway, incoming);
}
__device__ __forceinline__ v3 sample_microfacet(float roughness, v3 normal, v2 rn) {
    float phi = 2 * pif * rn.x;
    float theta = jl_atan(roughness * __builtin_sqrtf(rn.y / (1 - rn.y)));
    float sp, cp, st, ct;
    jl_sincos(phi, &sp, &cp);
    jl_sincos(theta, &st, &ct);
    v3 local = V3(cp * st, sp * st, ct);
    return normalize(mul(basis_fromz(normal), local));
}
__device__ __forceinline__ float sample_microfacet_pdf(float roughness, v3 normal, v3 halfway) {
    float cosine = dot(normal, halfway);
    if (cosine < 0) return 0;
    return microfacet_distribution(roughness, normal, halfway) * cosine;
}
__device__ __forceinline__ bool same_hemisphere(v3 normal, v3 outgoing, v3 incoming) {
    return dot(normal, outgoing) * dot(normal, incoming) >= 0;
}
__device__ __forceinline__ v3 splat(float s) { return V3(s, s, s); }

// ---------------------------------------------------------------- rough lobes (src/shading.jl)
__device__ __forceinline__ v3 eval_matte(v3 color, v3 n, v3 o, v3 i) {  // :14-19
    if (dot(n, i) * dot(n, o) <= 0) return V3(0, 0, 0);
    return (color / pif) * __builtin_fabsf(dot(n, i));
}
__device__ __forceinline__ float sample_matte_pdf(v3 n, v3 o, v3 i) {  // :26-37
    if (dot(n, i) * dot(n, o) <= 0) return 0;
    return sample_hemisphere_cos_pdf(up_normal(n, o), i);
}
__device__ __forceinline__ v3 eval_glossy(v3 color, float ior, float rough, v3 n, v3 o, v3 i) {  // :39-60
    if (dot(n, i) * dot(n, o) <= 0) return V3(0, 0, 0);
    v3 up = up_normal(n, o);
    float F1 = fresnel_dielectric(ior, up, o);
    v3 h = normalize(i + o);
    float F = fresnel_dielectric(ior, h, i);
    float D = microfacet_distribution(rough, up, h);
    float G = microfacet_shadowing(rough, up, h, o, i);
    float ci = __builtin_fabsf(dot(up, i));
    float spec = F * D * G / (4 * dot(up, o) * dot(up, i)) * ci;
    return ((color * (1 - F1)) / pif) * ci + splat(spec);
}
__device__ __forceinline__ v3 sample_glossy(float ior, float rough, v3 n, v3 o, float rnl, v2 rn) {  // :62-82
    v3 up = up_normal(n, o);
    if (rnl < fresnel_dielectric(ior, up, o)) {
        v3 h = sample_microfacet(rough, up, rn);
        v3 i = reflect(o, h);
        if (!same_hemisphere(up, o, i)) return V3(0, 0, 0);
        return i;
    }
    return sample_hemisphere_cos(up, rn);
}
__device__ __forceinline__ float sample_glossy_pdf(float ior, float rough, v3 n, v3 o, v3 i) {  // :84-101
    if (dot(n, i) * dot(n, o) <= 0) return 0;
    v3 up = up_normal(n, o);
    v3 h = normalize(o + i);
    float F = fresnel_dielectric(ior, up, o);
    return F * sample_microfacet_pdf(rough, up, h) / (4 * __builtin_fabsf(dot(o, h))) +
           (1 - F) * sample_hemisphere_cos_pdf(up, i);
}
__device__ __forceinline__ v3 eval_reflective(v3 color, float rough, v3 n, v3 o, v3 i) {  // :103-120
    if (dot(n, i) * dot(n, o) <= 0) return V3(0, 0, 0);
    v3 up = up_normal(n, o);
    v3 h = normalize(i + o);
    v3 F = fresnel_conductor(reflectivity_to_eta(color), h, i);
    float D = microfacet_distribution(rough, up, h);
    float G = microfacet_shadowing(rough, up, h, o, i);
    float den = 4 * dot(up, o) * dot(up, i);
    float ci = __builtin_fabsf(dot(up, i));
    return V3(F.x * D * G / den * ci, F.y * D * G / den * ci, F.z * D * G / den * ci);
}
__device__ __forceinline__ v3 sample_reflective(float rough, v3 n, v3 o, v2 rn) {  // :122-136
    v3 up = up_normal(n, o);
    v3 h = sample_microfacet(rough, up, rn);
    v3 i = reflect(o, h);
    if (!same_hemisphere(up, o, i)) return V3(0, 0, 0);
    return i;
}
__device__ __forceinline__ float sample_reflective_pdf(float rough, v3 n, v3 o, v3 i) {  // :138-151
    if (dot(n, i) * dot(n, o) <= 0) return 0;
    v3 up = up_normal(n, o);
    v3 h = normalize(o + i);
    return sample_microfacet_pdf(rough, up, h) / (4 * __builtin_fabsf(dot(o, h)));
}
__device__ __forceinline__ v3 eval_transparent(v3 color, float ior, float rough, v3 n, v3 o, v3 i) {  // :323-350
    v3 up = up_normal(n, o);
    if (dot(n, i) * dot(n, o) >= 0) {
        v3 h = normalize(i + o);
        float F = fresnel_dielectric(ior, h, o);
        float D = microfacet_distribution(rough, up, h);
        float G = microfacet_shadowing(rough, up, h, o, i);
        return splat(F * D * G / (4 * dot(up, o) * dot(up, i)) * __builtin_fabsf(dot(up, i)));
    }
    v3 refl = reflect(-i, up);
    v3 h = normalize(refl + o);
    float F = fresnel_dielectric(ior, h, o);
    float D = microfacet_distribution(rough, up, h);
    float G = microfacet_shadowing(rough, up, h, o, refl);
    float den = 4 * dot(up, o) * dot(up, refl);
    float cr = __builtin_fabsf(dot(up, refl));
    return V3(color.x * (1 - F) * D * G / den * cr, color.y * (1 - F) * D * G / den * cr,
              color.z * (1 - F) * D * G / den * cr);
}
__device__ __forceinline__ v3 sample_transparent(float ior, float rough, v3 n, v3 o, float rnl, v2 rn) {  // :352-377
    v3 up = up_normal(n, o);
    v3 h = sample_microfacet(rough, up, rn);
    if (rnl < fresnel_dielectric(ior, h, o)) {
        v3 i = reflect(o, h);
        if (!same_hemisphere(up, o, i)) return V3(0, 0, 0);
        return i;
    }
    v3 refl = reflect(o, h);
    v3 i = -reflect(refl, up);
    if (same_hemisphere(up, o, i)) return V3(0, 0, 0);
    return i;
}
__device__ __forceinline__ float sample_transparent_pdf(float ior, float rough, v3 n, v3 o, v3 i) {  // :379-401
    v3 up = up_normal(n, o);
    if (dot(n, i) * dot(n, o) >= 0) {
        v3 h = normalize(i + o);
        return fresnel_dielectric(ior, h, o) * sample_microfacet_pdf(rough, up, h) / (4 * __builtin_fabsf(dot(o, h)));
    }
    v3 refl = reflect(-i, up);
    v3 h = normalize(refl + o);
    float d = (1 - fresnel_dielectric(ior, h, o)) * sample_microfacet_pdf(rough, up, h);
    return d / (4 * __builtin_fabsf(dot(o, h)));
}
__device__ __forceinline__ v3 eval_refractive(float ior, float rough, v3 n, v3 o, v3 i) {  // :448-482
    bool entering = dot(n, o) >= 0;
    v3 up = entering ? n : -n;
    float rel_ior = entering ? ior : (1 / ior);
    if (dot(n, i) * dot(n, o) >= 0) {
        v3 h = normalize(i + o);
        float F = fresnel_dielectric(rel_ior, h, o);
        float D = microfacet_distribution(rough, up, h);
        float G = microfacet_shadowing(rough, up, h, o, i);
        return splat(F * D * G / __builtin_fabsf(4 * dot(n, o) * dot(n, i)) * __builtin_fabsf(dot(n, i)));
    }
    v3 h = (-normalize(i * rel_ior + o)) * (entering ? 1.0f : -1.0f);
    float F = fresnel_dielectric(rel_ior, h, o);
    float D = microfacet_distribution(rough, up, h);
    float G = microfacet_shadowing(rough, up, h, o, i);
    float a = __builtin_fabsf((dot(o, h) * dot(i, h)) / (dot(o, n) * dot(i, n)));
    float sq = rel_ior * dot(h, i) + dot(h, o);
    sq = sq * sq;  // ^2.0f0
    return splat(a * (1 - F) * D * G / sq * __builtin_fabsf(dot(n, i)));
}
__device__ __forceinline__ v3 sample_refractive(float ior, float rough, v3 n, v3 o, float rnl, v2 rn) {  // :484-509
    bool entering = dot(n, o) >= 0;
    v3 up = entering ? n : -n;
    v3 h = sample_microfacet(rough, up, rn);
    if (rnl < fresnel_dielectric(entering ? ior : (1 / ior), h, o)) {
        v3 i = reflect(o, h);
        if (!same_hemisphere(up, o, i)) return V3(0, 0, 0);
        return i;
    }
    v3 i = refract(o, h, entering ? (1 / ior) : ior);
    if (same_hemisphere(up, o, i)) return V3(0, 0, 0);
    return i;
}
__device__ __forceinline__ float sample_refractive_pdf(float ior, float rough, v3 n, v3 o, v3 i) {  // :511-534
    bool entering = dot(n, o) >= 0;
    v3 up = entering ? n : -n;
    float rel_ior = entering ? ior : (1 / ior);
    if (dot(n, i) * dot(n, o) >= 0) {
        v3 h = normalize(i + o);
        return fresnel_dielectric(rel_ior, h, o) * sample_microfacet_pdf(rough, up, h) /
               (4 * __builtin_fabsf(dot(o, h)));
    }
    v3 h = (-normalize(i * rel_ior + o)) * (entering ? 1.0f : -1.0f);
    float sq = rel_ior * dot(h, i) + dot(h, o);
    sq = sq * sq;
    return (1 - fresnel_dielectric(rel_ior, h, o)) * sample_microfacet_pdf(rough, up, h) *
           __builtin_fabsf(dot(h, i)) / sq;
}

// ---------------------------------------------------------------- delta lobes (src/shading.jl)
__device__ __forceinline__ v3 eval_reflective_delta(v3 color, v3 n, v3 o, v3 i) {  // :202-213
    if (dot(n, i) * dot(n, o) <= 0) return V3(0, 0, 0);
    return fresnel_conductor(reflectivity_to_eta(color), up_normal(n, o), o);
}
__device__ __forceinline__ v3 eval_transparent_delta(v3 color, float ior, v3 n, v3 o, v3 i) {  // :403-416
    v3 up = up_normal(n, o);
    if (dot(n, i) * dot(n, o) >= 0) return splat(fresnel_dielectric(ior, up, o));
    return color * (1 - fresnel_dielectric(ior, up, o));
}
__device__ __forceinline__ v3 sample_transparent_delta(float ior, v3 n, v3 o, float rnl) {  // :418-431
    v3 up = up_normal(n, o);
    if (rnl < fresnel_dielectric(ior, up, o)) return reflect(o, up);
    return -o;
}
__device__ __forceinline__ float sample_transparent_delta_pdf(float ior, v3 n, v3 o, v3 i) {  // :433-446
    v3 up = up_normal(n, o);
    if (dot(n, i) * dot(n, o) >= 0) return fresnel_dielectric(ior, up, o);
    return 1 - fresnel_dielectric(ior, up, o);
}
__device__ __forceinline__ v3 eval_refractive_delta(float ior, v3 n, v3 o, v3 i) {  // :536-560
    if ((double)__builtin_fabsf(ior - 1) < 1e-3) return dot(n, i) * dot(n, o) <= 0 ? V3(1, 1, 1) : V3(0, 0, 0);
    bool entering = dot(n, o) >= 0;
    v3 up = entering ? n : -n;
    float rel_ior = entering ? ior : (1 / ior);
    if (dot(n, i) * dot(n, o) >= 0) return splat(fresnel_dielectric(rel_ior, up, o));
    return splat((1 / (rel_ior * rel_ior)) * (1 - fresnel_dielectric(rel_ior, up, o)));
}
__device__ __forceinline__ v3 sample_refractive_delta(float ior, v3 n, v3 o, float rnl) {  // :562-580
    if ((double)__builtin_fabsf(ior - 1) < 1e-3) return -o;
    bool entering = dot(n, o) >= 0;
    v3 up = entering ? n : -n;
    float rel_ior = entering ? ior : (1 / ior);
    if (rnl < fresnel_dielectric(rel_ior, up, o)) return reflect(o, up);
    return refract(o, up, 1 / rel_ior);
}
__device__ __forceinline__ float sample_refractive_delta_pdf(float ior, v3 n, v3 o, v3 i) {  // :582-604
    if (__builtin_fabsf(ior - 1) < 0.001f) return dot(n, i) * dot(n, o) < 0 ? 1.0f : 0.0f;
    bool entering = dot(n, o) >= 0;
    v3 up = entering ? n : -n;
    float rel_ior = entering ? ior : (1 / ior);
    if (dot(n, i) * dot(n, o) >= 0) return fresnel_dielectric(rel_ior, up, o);
    return 1 - fresnel_dielectric(rel_ior, up, o);
}

// ---------------------------------------------------------------- dispatch (src/trace.jl)
// The dispatchers take the kernel's scene feature bits (jt_device.h): without FT_VOL a scene has
// no refractive/subsurface/volumetric material, so those cases are unreachable and compiled out.
template <int F>
__device__ __forceinline__ v3 eval_bsdfcos(const MatPoint& m, v3 n, v3 o, v3 i) {  // :692-755
    if (m.roughness == 0) return V3(0, 0, 0);
    switch (m.type) {
        case M_MATTE: return eval_matte(m.color, n, o, i);
        case M_GLOSSY: return eval_glossy(m.color, m.ior, m.roughness, n, o, i);
        case M_REFLECTIVE: return eval_reflective(m.color, m.roughness, n, o, i);
        case M_TRANSPARENT: return eval_transparent(m.color, m.ior, m.roughness, n, o, i);
        case M_REFRACTIVE:
        case M_SUBSURFACE: return (F & FT_VOL) ? eval_refractive(m.ior, m.roughness, n, o, i) : V3(0, 0, 0);
        default: return V3(0, 0, 0);
    }
}
template <int F>
__device__ __forceinline__ v3 sample_bsdfcos(const MatPoint& m, v3 n, v3 o, float rnl, v2 rn) {  // :780-849
    if (m.roughness == 0) return V3(0, 0, 0);
    switch (m.type) {
        case M_MATTE: return sample_hemisphere_cos(up_normal(n, o), rn);
        case M_GLOSSY: return sample_glossy(m.ior, m.roughness, n, o, rnl, rn);
        case M_REFLECTIVE: return sample_reflective(m.roughness, n, o, rn);
        case M_TRANSPARENT: return sample_transparent(m.ior, m.roughness, n, o, rnl, rn);
        case M_REFRACTIVE:
        case M_SUBSURFACE: return (F & FT_VOL) ? sample_refractive(m.ior, m.roughness, n, o, rnl, rn) : V3(0, 0, 0);
        default: return V3(0, 0, 0);
    }
}
template <int F>
__device__ __forceinline__ float sample_bsdfcos_pdf(const MatPoint& m, v3 n, v3 o, v3 i) {  // :874-943
    if (m.roughness == 0) return 0;
    switch (m.type) {
        case M_MATTE: return sample_matte_pdf(n, o, i);
        case M_GLOSSY: return sample_glossy_pdf(m.ior, m.roughness, n, o, i);
        case M_REFLECTIVE: return sample_reflective_pdf(m.roughness, n, o, i);
        case M_TRANSPARENT: return sample_transparent_pdf(m.ior, m.roughness, n, o, i);
        case M_REFRACTIVE:
        case M_SUBSURFACE: return (F & FT_VOL) ? sample_refractive_pdf(m.ior, m.roughness, n, o, i) : 0.0f;
        default: return 0;
    }
}
// eval_bsdfcos and sample_bsdfcos_pdf of one (material, n, o, i), evaluated in ONE branch per
// material type (material-keyed shading): the two reference functions run back to back
// on every non-delta bounce (src/trace.jl:386-392); as two switches a wave executes each present
// type's code region twice, once per switch; here once, and the compiler shares what the two compute
// alike (dot products, Fresnel terms, the GGX distribution). The same float operations in the same
// order per function, so results are unchanged.
template <int F>
__device__ __forceinline__ void eval_bsdfcos_pdf(const MatPoint& m, v3 n, v3 o, v3 i, v3& f, float& pdf) {
    f = V3(0, 0, 0);
    pdf = 0;
    if (m.roughness == 0) return;
    switch (m.type) {
        case M_MATTE:
            f = eval_matte(m.color, n, o, i);
            pdf = sample_matte_pdf(n, o, i);
            return;
        case M_GLOSSY:
            f = eval_glossy(m.color, m.ior, m.roughness, n, o, i);
            pdf = sample_glossy_pdf(m.ior, m.roughness, n, o, i);
            return;
        case M_REFLECTIVE:
            f = eval_reflective(m.color, m.roughness, n, o, i);
            pdf = sample_reflective_pdf(m.roughness, n, o, i);
            return;
        case M_TRANSPARENT:
            f = eval_transparent(m.color, m.ior, m.roughness, n, o, i);
            pdf = sample_transparent_pdf(m.ior, m.roughness, n, o, i);
            return;
        case M_REFRACTIVE:
        case M_SUBSURFACE:
            if (F & FT_VOL) {
                f = eval_refractive(m.ior, m.roughness, n, o, i);
                pdf = sample_refractive_pdf(m.ior, m.roughness, n, o, i);
            }
            return;
        default: return;
    }
}
template <int F>
__device__ __forceinline__ v3 eval_delta(const MatPoint& m, v3 n, v3 o, v3 i) {  // :757-778
    if (m.roughness != 0) return V3(0, 0, 0);
    switch (m.type) {
        case M_REFLECTIVE: return eval_reflective_delta(m.color, n, o, i);
        case M_TRANSPARENT: return eval_transparent_delta(m.color, m.ior, n, o, i);
        case M_REFRACTIVE: return (F & FT_VOL) ? eval_refractive_delta(m.ior, n, o, i) : V3(0, 0, 0);
        case M_VOLUMETRIC:  // passthrough
            return ((F & FT_VOL) && !(dot(n, i) * dot(n, o) >= 0)) ? V3(1, 1, 1) : V3(0, 0, 0);
        default: return V3(0, 0, 0);
    }
}
template <int F>
__device__ __forceinline__ v3 sample_delta(const MatPoint& m, v3 n, v3 o, float rnl) {  // :851-872
    if (m.roughness != 0) return V3(0, 0, 0);
    switch (m.type) {
        case M_REFLECTIVE: return reflect(o, up_normal(n, o));
        case M_TRANSPARENT: return sample_transparent_delta(m.ior, n, o, rnl);
        case M_REFRACTIVE: return (F & FT_VOL) ? sample_refractive_delta(m.ior, n, o, rnl) : V3(0, 0, 0);
        case M_VOLUMETRIC: return -o;
        default: return V3(0, 0, 0);
    }
}
template <int F>
__device__ __forceinline__ float sample_delta_pdf(const MatPoint& m, v3 n, v3 o, v3 i) {  // :945-966
    if (m.roughness != 0) return 0;
    switch (m.type) {
        case M_REFLECTIVE: return dot(n, i) * dot(n, o) <= 0 ? 0.0f : 1.0f;
        case M_TRANSPARENT: return sample_transparent_delta_pdf(m.ior, n, o, i);
        case M_REFRACTIVE: return (F & FT_VOL) ? sample_refractive_delta_pdf(m.ior, n, o, i) : 0.0f;
        case M_VOLUMETRIC: return dot(n, i) * dot(n, o) >= 0 ? 0.0f : 1.0f;
        default: return 0;
    }
}
__device__ __forceinline__ bool is_delta(const MatPoint& m) {  // src/scene.jl:916-920
    return (m.type == M_REFLECTIVE && m.roughness == 0) || (m.type == M_REFRACTIVE && m.roughness == 0) ||
           (m.type == M_TRANSPARENT && m.roughness == 0) || (m.type == M_VOLUMETRIC);
}

// ---------------------------------------------------------------- volumes (src/shading.jl:648-693)
struct Volume {
    v3 density, scattering;
    float scanisotropy;
};
__device__ __forceinline__ v3 eval_transmittance(v3 density, float distance) {
    return V3(jl_exp(-density.x * distance), jl_exp(-density.y * distance), jl_exp(-density.z * distance));
}
__device__ __forceinline__ float sample_transmittance(v3 density, float max_distance, float rl, float rd) {
    int channel = jl_clampi((int)__builtin_truncf(rl * 3), 1, 3);  // reference bias: channel 3 unreachable
    float dc = channel == 1 ? density.x : (channel == 2 ? density.y : density.z);
    float distance = dc == 0 ? __builtin_inff() : -jl_log(1 - rd) / dc;
    return jl_min(distance, max_distance);
}
__device__ __forceinline__ float sample_transmittance_pdf(v3 density, float distance, float max_distance) {
    if (distance < max_distance)
        return ((density.x * jl_exp(-density.x * distance) + density.y * jl_exp(-density.y * distance)) +
                density.z * jl_exp(-density.z * distance)) /
               3;
    return ((jl_exp(-density.x * max_distance) + jl_exp(-density.y * max_distance)) +
            jl_exp(-density.z * max_distance)) /
           3;
}
__device__ __forceinline__ float eval_phasefunction(float an, v3 o, v3 i) {
    float cosine = -dot(o, i);
    float denom = 1 + an * an - 2 * an * cosine;
    return (1 - an * an) / (4 * pif * denom * __builtin_sqrtf(denom));
}
__device__ __forceinline__ v3 sample_phasefunction(float an, v3 o, v2 rn) {
    float cos_theta;
    if (__builtin_fabsf(an) < 0.001f) {
        cos_theta = 1 - 2 * rn.y;
    } else {
        float square = (1 - an * an) / (1 + an - 2 * an * rn.y);
        cos_theta = (1 + an * an - square * square) / (2 * an);
    }
    float sin_theta = __builtin_sqrtf(jl_max(0.0f, 1 - cos_theta * cos_theta));
    float phi = 2 * pif * rn.x;
    float s, c;
    jl_sincos(phi, &s, &c);
    v3 local = V3(sin_theta * c, sin_theta * s, cos_theta);
    return mul(basis_fromz(-o), local);
}
// eval_scattering / sample_scattering(_pdf) (src/trace.jl:1086-1115)
__device__ __forceinline__ v3 eval_scattering(const Volume& m, v3 o, v3 i) {
    if (is_zero(m.density)) return V3(0, 0, 0);
    return (m.scattering * m.density) * eval_phasefunction(m.scanisotropy, o, i);
}
__device__ __forceinline__ v3 sample_scattering(const Volume& m, v3 o, v2 rn) {
    if (is_zero(m.density)) return V3(0, 0, 0);
    return sample_phasefunction(m.scanisotropy, o, rn);
}
__device__ __forceinline__ float sample_scattering_pdf(const Volume& m, v3 o, v3 i) {
    if (is_zero(m.density)) return 0;
    return eval_phasefunction(m.scanisotropy, o, i);
}

}  // namespace jtd
