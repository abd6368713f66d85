// jt_internal.h — shared host-side helpers of libjtrace_hip (not part of the ABI).
#pragma once

#include <cmath>
#include <cstdint>
#include <map>
#include <string>

#include "../../include/jtrace.h"

namespace jt {

// thread-local last error (jt_last_error)
void set_error(const std::string& msg);
int fail(int status, const std::string& msg);

// run-time options set through jt_set_option (include/jtrace.h), never read from the environment:
// a copy of the process-wide table, taken once by jt_create / jt_create_multi
std::map<std::string, std::string> options_snapshot();

// Julia float semantics used by the host restatements (base/math.jl, Julia 1.8):
// NaN-propagating, signbit-aware min/max; clamp = ifelse(x > hi, hi, ifelse(x < lo, lo, x)).
inline float jl_min(float x, float y) {
    bool c = (y < x) || (std::signbit(y) && !std::signbit(x));
    return c ? (std::isnan(x) ? x : y) : (std::isnan(y) ? y : x);
}
inline float jl_max(float x, float y) {
    bool c = (y > x) || (!std::signbit(y) && std::signbit(x));
    return c ? (std::isnan(x) ? x : y) : (std::isnan(y) ? y : x);
}

struct f3 {
    float x, y, z;
};
inline f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
inline f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
inline f3 operator/(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
inline f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }
inline float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline f3 cross(f3 a, f3 b) {
    return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float length(f3 a) { return std::sqrt(dot(a, a)); }
// normalize (src/math.jl:71-78) — the same float operations as the device version
inline f3 normalize(f3 a) {
    const float l = std::sqrt(dot(a, a));
    return l != 0 ? a / l : a;
}
inline float comp(f3 v, int axis) { return axis == 0 ? v.x : (axis == 1 ? v.y : v.z); }

// Frame3f: columns x, y, z, o (src/math.jl:46)
struct frame3 {
    f3 x, y, z, o;
};
inline frame3 load_frame(const float* a) {
    return frame3{mk3(a[0], a[1], a[2]), mk3(a[3], a[4], a[5]), mk3(a[6], a[7], a[8]),
                  mk3(a[9], a[10], a[11])};
}
inline void store_frame(const frame3& f, float* a) {
    const float v[12] = {f.x.x, f.x.y, f.x.z, f.y.x, f.y.y, f.y.z,
                         f.z.x, f.z.y, f.z.z, f.o.x, f.o.y, f.o.z};
    for (int k = 0; k < 12; k++) a[k] = v[k];
}
// transform_point (src/math.jl:80-81)
inline f3 transform_point(const frame3& f, f3 p) { return ((f.x * p.x + f.y * p.y) + f.z * p.z) + f.o; }
// transform_vector (src/math.jl:83-84)
inline f3 transform_vector(const frame3& f, f3 b) { return (f.x * b.x + f.y * b.y) + f.z * b.z; }
// inverse(frame, non_rigid) (src/math.jl:95-117)
frame3 inverse_frame(const frame3& f, bool non_rigid);

}  // namespace jt
