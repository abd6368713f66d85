// jt_host.cpp — host helpers of the C-ABI: errors, version, BVH build, trace lights, image size.
//
// These restate the reference's host-side code the hot path consumes (the reference keeps them
// in Julia; the drop-in's Julia shim may pass its own). Node order, primitive permutation and
// every float operation follow src/bvh.jl so traversal order and hit tie-breaking match.
// Compiled with -ffp-contract=off (no FMA contraction, as Julia without muladd).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "jt_internal.h"

namespace jt {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int status, const std::string& msg) {
    set_error(msg);
    return status;
}

// The run-time options of include/jtrace.h (jt_set_option). Process-wide; jt_create reads a copy.
static std::mutex g_opt_mu;
static std::map<std::string, std::string> g_opts;
static const char* const kOptionNames[] = {
    "env_alias",  "features",    "lds_scene",   "lds_stack",  "light_inline", "streams",
    "wait_lanes", "light_lanes", "multi_split", "tile_share",  "test_lds_ring",
};
std::map<std::string, std::string> options_snapshot() {
    std::lock_guard<std::mutex> g(g_opt_mu);
    return g_opts;
}

frame3 inverse_frame(const frame3& f, bool non_rigid) {
    // rotation(frame) columns
    f3 c1 = f.x, c2 = f.y, c3 = f.z;
    f3 m1, m2, m3;  // columns of minv
    if (non_rigid) {
        // inverse(m) = adjoint(m) * (1 / determinant(m)); adjoint = transpose(cofactor columns)
        f3 k1 = cross(c2, c3), k2 = cross(c3, c1), k3 = cross(c1, c2);
        f3 a1 = mk3(k1.x, k2.x, k3.x), a2 = mk3(k1.y, k2.y, k3.y), a3 = mk3(k1.z, k2.z, k3.z);
        float det = dot(c1, cross(c2, c3));
        float s = 1.0f / det;
        m1 = a1 * s;
        m2 = a2 * s;
        m3 = a3 * s;
    } else {
        m1 = mk3(c1.x, c2.x, c3.x);
        m2 = mk3(c1.y, c2.y, c3.y);
        m3 = mk3(c1.z, c2.z, c3.z);
    }
    f3 t = (m1 * f.o.x + m2 * f.o.y) + m3 * f.o.z;  // Base.:*(m::Mat3f, f::Vec3f)
    return frame3{m1, m2, m3, -t};
}

// ----------------------------------------------------------------------------- BVH (src/bvh.jl)
struct bbox {
    f3 mn, mx;
};
static inline bbox empty_bbox() {  // Bbox3f() (src/geometry.jl:26-29)
    const float inf = INFINITY;
    return bbox{mk3(inf, inf, inf), mk3(-inf, -inf, -inf)};
}
static inline bbox merge(const bbox& b, f3 p) {  // merge_bbox3f(bbox, point)
    return bbox{mk3(jl_min(b.mn.x, p.x), jl_min(b.mn.y, p.y), jl_min(b.mn.z, p.z)),
                mk3(jl_max(b.mx.x, p.x), jl_max(b.mx.y, p.y), jl_max(b.mx.z, p.z))};
}
static inline bbox merge(const bbox& a, const bbox& b) {  // merge_bbox3f(bbox, bbox)
    return bbox{mk3(jl_min(a.mn.x, b.mn.x), jl_min(a.mn.y, b.mn.y), jl_min(a.mn.z, b.mn.z)),
                mk3(jl_max(a.mx.x, b.mx.x), jl_max(a.mx.y, b.mx.y), jl_max(a.mx.z, b.mx.z))};
}
static inline f3 center(const bbox& b) { return (b.mn + b.mx) / 2.0f; }
static inline float bbox_area(const bbox& b) {  // src/bvh.jl:276-279
    f3 s = b.mx - b.mn;
    return ((0.000000000001f + 2 * s.x * s.y) + 2 * s.x * s.z) + 2 * s.y * s.z;
}

struct Builder {
    const std::vector<bbox>& boxes;
    bool hq;
    std::vector<int32_t> prims;
    std::vector<f3> centers;
    std::vector<jt_bvh_node> nodes;

    explicit Builder(const std::vector<bbox>& b, bool high_quality) : boxes(b), hq(high_quality) {}

    // partition (src/bvh.jl:281-304), 0-based inclusive range; may return start - 1
    long partition(int axis, float split, long start, long stop) {
        long i = start, j = stop;
        for (;;) {
            while (i <= stop && comp(centers[prims[i]], axis) < split) i++;
            while (j >= start && comp(centers[prims[j]], axis) >= split) j--;
            if (i >= j) break;
            std::swap(prims[i], prims[j]);
        }
        return j;
    }
    bbox centroid_box(long left, long right) const {
        bbox cb = empty_bbox();
        for (long i = left; i <= right; i++) cb = merge(cb, centers[prims[i]]);
        return cb;
    }
    // split_middle (src/bvh.jl:185-216) -> (last index of the left child, axis)
    void split_middle(long left, long right, long& mid, int& axis) {
        bbox cb = centroid_box(left, right);
        f3 cs = cb.mx - cb.mn;
        if (cs.x == 0 && cs.y == 0 && cs.z == 0) {
            mid = (left + right + 1) / 2;  // div(l+r+1, 2) in 1-based terms, minus 1
            axis = 0;
            return;
        }
        axis = 0;
        if (cs.x >= cs.y && cs.x >= cs.z) axis = 0;
        if (cs.y >= cs.x && cs.y >= cs.z) axis = 1;
        if (cs.z >= cs.x && cs.z >= cs.y) axis = 2;
        float split = comp(center(cb), axis);
        long m = partition(axis, split, left, right);
        mid = (m < left || m > right) ? (left + right + 1) / 2 : m;
    }
    // split_sah (src/bvh.jl:218-274), 16 bins per axis
    void split_sah(long left, long right, long& mid, int& axis) {
        bbox cb = centroid_box(left, right);
        f3 cs = cb.mx - cb.mn;
        if (cs.x == 0 && cs.y == 0 && cs.z == 0) {
            mid = (left + right + 1) / 2;
            axis = 0;
            return;
        }
        axis = 0;
        const int nbins = 16;
        float split = 0.0f, min_cost = INFINITY;
        const float carea = bbox_area(cb);
        for (int sa = 0; sa < 3; sa++) {
            for (int b = 1; b < nbins; b++) {
                float bsplit = comp(cb.mn, sa) + (float)b * comp(cs, sa) / (float)nbins;
                bbox lb = empty_bbox(), rb = empty_bbox();
                long ln = 0, rn = 0;
                for (long i = left; i <= right; i++) {
                    if (comp(centers[prims[i]], sa) < bsplit) {
                        lb = merge(lb, boxes[prims[i]]);
                        ln++;
                    } else {
                        rb = merge(rb, boxes[prims[i]]);
                        rn++;
                    }
                }
                float cost = (1 + (float)ln * bbox_area(lb) / carea) + (float)rn * bbox_area(rb) / carea;
                if (cost < min_cost) {
                    min_cost = cost;
                    split = bsplit;
                    axis = sa;
                }
            }
        }
        long m = partition(axis, split, left, right);
        mid = (m == left || m == right) ? (left + right + 1) / 2 : m;
    }
    // make_bvh (src/bvh.jl:138-183): LIFO work stack, children allocated in pairs
    void build() {
        const long n = (long)boxes.size();
        prims.resize(n);
        centers.resize(n);
        for (long i = 0; i < n; i++) {
            prims[i] = (int32_t)i;
            centers[i] = center(boxes[i]);
        }
        struct Item {
            long node, left, right;
        };
        std::vector<Item> stack;
        std::vector<bbox> nb;
        nodes.reserve(2 * n + 1);
        nb.reserve(2 * n + 1);
        nodes.push_back(jt_bvh_node{});
        nb.push_back(empty_bbox());
        stack.push_back(Item{0, 0, n - 1});
        while (!stack.empty()) {
            Item it = stack.back();
            stack.pop_back();
            bbox b = nb[it.node];
            for (long i = it.left; i <= it.right; i++) b = merge(b, boxes[prims[i]]);
            nb[it.node] = b;
            if (it.right - it.left + 1 > 4) {  // BVH_MAX_PRIMS = 4 (src/bvh.jl:32)
                long mid;
                int axis;
                if (hq) split_sah(it.left, it.right, mid, axis);
                else split_middle(it.left, it.right, mid, axis);
                long start = (long)nodes.size();
                jt_bvh_node& nd = nodes[it.node];
                nd.start = (int32_t)start;
                nd.num = 2;
                nd.axis = (int8_t)axis;
                nd.internal = 1;
                nodes.push_back(jt_bvh_node{});
                nodes.push_back(jt_bvh_node{});
                nb.push_back(empty_bbox());
                nb.push_back(empty_bbox());
                stack.push_back(Item{start, it.left, mid});
                stack.push_back(Item{start + 1, mid + 1, it.right});
            } else {
                jt_bvh_node& nd = nodes[it.node];
                nd.start = (int32_t)it.left;
                nd.num = (int16_t)(it.right - it.left + 1);
                nd.internal = 0;
            }
        }
        for (size_t k = 0; k < nodes.size(); k++) {
            nodes[k].bmin[0] = nb[k].mn.x;
            nodes[k].bmin[1] = nb[k].mn.y;
            nodes[k].bmin[2] = nb[k].mn.z;
            nodes[k].bmax[0] = nb[k].mx.x;
            nodes[k].bmax[1] = nb[k].mx.y;
            nodes[k].bmax[2] = nb[k].mx.z;
        }
    }
};

static int export_tree(Builder& b, jt_bvh_tree* out) {
    out->nnodes = (int32_t)b.nodes.size();
    out->nprimitives = (int32_t)b.prims.size();
    out->nodes = (jt_bvh_node*)std::malloc(sizeof(jt_bvh_node) * std::max<size_t>(1, b.nodes.size()));
    out->primitives = (int32_t*)std::malloc(sizeof(int32_t) * std::max<size_t>(1, b.prims.size()));
    if (!out->nodes || !out->primitives) return JT_ERR_NOMEM;
    std::memcpy(out->nodes, b.nodes.data(), sizeof(jt_bvh_node) * b.nodes.size());
    std::memcpy(out->primitives, b.prims.data(), sizeof(int32_t) * b.prims.size());
    return JT_OK;
}

static inline f3 vpos(const jt_shape& s, int32_t v) {
    return mk3(s.positions[3 * v], s.positions[3 * v + 1], s.positions[3 * v + 2]);
}

// make_shape_bvh (src/bvh.jl:90-136): element bounds then make_bvh
static int build_shape(const jt_shape& s, bool hq, jt_bvh_tree* out, std::string& err) {
    std::vector<bbox> boxes;
    if (s.ntriangles > 0) {
        boxes.resize(s.ntriangles);
        for (int32_t i = 0; i < s.ntriangles; i++) {
            const int32_t* t = &s.triangles[3 * i];
            f3 a = vpos(s, t[0]), b = vpos(s, t[1]), c = vpos(s, t[2]);
            // triangle_bounds = Bbox3f(min.(p1, p2, p3), max.(p1, p2, p3)) (src/geometry.jl:64)
            boxes[i] = bbox{mk3(jl_min(jl_min(a.x, b.x), c.x), jl_min(jl_min(a.y, b.y), c.y),
                                jl_min(jl_min(a.z, b.z), c.z)),
                            mk3(jl_max(jl_max(a.x, b.x), c.x), jl_max(jl_max(a.y, b.y), c.y),
                                jl_max(jl_max(a.z, b.z), c.z))};
        }
    } else if (s.nquads > 0) {
        boxes.resize(s.nquads);
        for (int32_t i = 0; i < s.nquads; i++) {
            const int32_t* q = &s.quads[4 * i];
            f3 a = vpos(s, q[0]), b = vpos(s, q[1]), c = vpos(s, q[2]), d = vpos(s, q[3]);
            boxes[i] = bbox{mk3(jl_min(jl_min(jl_min(a.x, b.x), c.x), d.x),
                                jl_min(jl_min(jl_min(a.y, b.y), c.y), d.y),
                                jl_min(jl_min(jl_min(a.z, b.z), c.z), d.z)),
                            mk3(jl_max(jl_max(jl_max(a.x, b.x), c.x), d.x),
                                jl_max(jl_max(jl_max(a.y, b.y), c.y), d.y),
                                jl_max(jl_max(jl_max(a.z, b.z), c.z), d.z))};
        }
    } else {
        err = "shape without triangles or quads (points/lines are not shaded by the reference, "
              "src/scene.jl:429,605; an empty shape throws in make_shape_bvh)";
        return JT_ERR_UNSUPPORTED;
    }
    Builder b(boxes, hq);
    b.build();
    return export_tree(b, out);
}

}  // namespace jt

using namespace jt;

extern "C" {

#ifndef JT_SOURCE_HASH
#define JT_SOURCE_HASH "unknown"
#endif
// ABI version and the source hash of this build (scripts/roofline.py source_hash)
#define JT_STR2(x) #x
#define JT_STR(x) JT_STR2(x)
const char* jt_version(void) { return "jtrace-mi355x 0.4 (gfx950 HIP, ABI " JT_STR(JT_ABI_VERSION) ", source " JT_SOURCE_HASH ")"; }
int jt_abi_version(void) { return JT_ABI_VERSION; }
const char* jt_last_error(void) { return jt::g_last_error.c_str(); }

int jt_set_option(const char* name, const char* value) {
    std::lock_guard<std::mutex> g(jt::g_opt_mu);
    if (!name) {
        if (value) return fail(JT_ERR_INVALID, "jt_set_option: a value without a name");
        jt::g_opts.clear();
        return JT_OK;
    }
    bool known = false;
    for (const char* k : jt::kOptionNames) known = known || std::strcmp(k, name) == 0;
    if (!known) return fail(JT_ERR_INVALID, std::string("jt_set_option: unknown option '") + name + "'");
    if (value) jt::g_opts[name] = value;
    else jt::g_opts.erase(name);
    return JT_OK;
}

static int validate_scene(const jt_scene* scene) {
    if (!scene) return fail(JT_ERR_INVALID, "scene is NULL");
    for (int32_t i = 0; i < scene->ninstances; i++) {
        const jt_instance& in = scene->instances[i];
        if (in.shape < 0 || in.shape >= scene->nshapes)
            return fail(JT_ERR_INVALID, "instance " + std::to_string(i) + " has an invalid shape id");
        if (in.material < 0 || in.material >= scene->nmaterials)
            return fail(JT_ERR_INVALID, "instance " + std::to_string(i) + " has an invalid material id");
    }
    for (int32_t s = 0; s < scene->nshapes; s++) {
        const jt_shape& sh = scene->shapes[s];
        const int32_t* idx = sh.ntriangles ? sh.triangles : sh.quads;
        long n = sh.ntriangles ? 3L * sh.ntriangles : 4L * sh.nquads;
        for (long k = 0; k < n; k++)
            if (idx[k] < 0 || idx[k] >= sh.npositions)
                return fail(JT_ERR_INVALID, "shape " + std::to_string(s) + " has an out-of-range vertex id");
    }
    return JT_OK;
}

int jt_build_scene_bvh(const jt_scene* scene, int32_t high_quality, jt_scene_bvh* out) {
    if (!out) return fail(JT_ERR_INVALID, "out is NULL");
    std::memset(out, 0, sizeof(*out));
    int st = validate_scene(scene);
    if (st != JT_OK) return st;
    out->nshapes = scene->nshapes;
    out->blas = (jt_bvh_tree*)std::calloc(std::max(1, scene->nshapes), sizeof(jt_bvh_tree));
    if (!out->blas) return fail(JT_ERR_NOMEM, "out of host memory");
    // per-shape builds are independent (the reference threads them, src/bvh.jl:73)
    std::vector<int> status(scene->nshapes, JT_OK);
    std::vector<std::string> errs(scene->nshapes);
    unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (scene->nshapes < 64) nth = 1;
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nth; t++) {
        auto work = [&, t]() {
            for (int32_t s = (int32_t)t; s < scene->nshapes; s += (int32_t)nth)
                status[s] = build_shape(scene->shapes[s], high_quality != 0, &out->blas[s], errs[s]);
        };
        if (nth == 1) work();
        else pool.emplace_back(work);
    }
    for (auto& th : pool) th.join();
    for (int32_t s = 0; s < scene->nshapes; s++) {
        if (status[s] != JT_OK) {
            std::string e = "shape " + std::to_string(s) + ": " + errs[s];
            jt_free_scene_bvh(out);
            return fail(status[s], e);
        }
    }
    // instance bounds: transform_bbox(frame, root box) (src/bvh.jl:77-85, src/geometry.jl:70-86)
    std::vector<bbox> boxes(scene->ninstances);
    for (int32_t i = 0; i < scene->ninstances; i++) {
        const jt_instance& in = scene->instances[i];
        const jt_bvh_tree& t = out->blas[in.shape];
        if (t.nnodes == 0) {
            boxes[i] = empty_bbox();
            continue;
        }
        const jt_bvh_node& r = t.nodes[0];
        frame3 f = load_frame(in.frame);
        const f3 corners[8] = {mk3(r.bmin[0], r.bmin[1], r.bmin[2]), mk3(r.bmin[0], r.bmin[1], r.bmax[2]),
                               mk3(r.bmin[0], r.bmax[1], r.bmin[2]), mk3(r.bmin[0], r.bmax[1], r.bmax[2]),
                               mk3(r.bmax[0], r.bmin[1], r.bmin[2]), mk3(r.bmax[0], r.bmin[1], r.bmax[2]),
                               mk3(r.bmax[0], r.bmax[1], r.bmin[2]), mk3(r.bmax[0], r.bmax[1], r.bmax[2])};
        bbox x = empty_bbox();
        for (const f3& c : corners) x = merge(x, transform_point(f, c));
        boxes[i] = x;
    }
    Builder tl(boxes, high_quality != 0);
    tl.build();
    st = export_tree(tl, &out->tlas);
    if (st != JT_OK) {
        jt_free_scene_bvh(out);
        return fail(st, "out of host memory");
    }
    return JT_OK;
}

void jt_free_scene_bvh(jt_scene_bvh* bvh) {
    if (!bvh) return;
    std::free(bvh->tlas.nodes);
    std::free(bvh->tlas.primitives);
    if (bvh->blas)
        for (int32_t s = 0; s < bvh->nshapes; s++) {
            std::free(bvh->blas[s].nodes);
            std::free(bvh->blas[s].primitives);
        }
    std::free(bvh->blas);
    std::memset(bvh, 0, sizeof(*bvh));
}

// triangle_area / quad_area (src/geometry.jl:264-271)
static inline float triangle_area(f3 p0, f3 p1, f3 p2) { return length(cross(p1 - p0, p2 - p0)) / 2; }
static inline float quad_area(f3 p0, f3 p1, f3 p2, f3 p3) {
    return triangle_area(p0, p1, p3) + triangle_area(p2, p3, p1);
}

// make_trace_lights (src/trace.jl:117-187)
int jt_make_lights(const jt_scene* scene, jt_lights* out) {
    if (!out) return fail(JT_ERR_INVALID, "out is NULL");
    std::memset(out, 0, sizeof(*out));
    int st = validate_scene(scene);
    if (st != JT_OK) return st;
    std::vector<jt_light> lights;
    auto cleanup = [&]() {
        for (auto& l : lights) std::free(l.cdf);
    };
    for (int32_t h = 0; h < scene->ninstances; h++) {
        const jt_instance& in = scene->instances[h];
        const jt_material& m = scene->materials[in.material];
        if (m.emission[0] == 0 && m.emission[1] == 0 && m.emission[2] == 0) continue;
        const jt_shape& s = scene->shapes[in.shape];
        if (s.ntriangles == 0 && s.nquads == 0) continue;
        jt_light l{h, -1, 0, nullptr};
        const bool quads = s.nquads != 0;  // the quad CDF overwrites the triangle one (:146-160)
        l.ncdf = quads ? s.nquads : s.ntriangles;
        l.cdf = (float*)std::malloc(sizeof(float) * l.ncdf);
        if (!l.cdf) {
            cleanup();
            return fail(JT_ERR_NOMEM, "out of host memory");
        }
        for (int32_t i = 0; i < l.ncdf; i++) {
            if (quads) {
                const int32_t* q = &s.quads[4 * i];
                l.cdf[i] = quad_area(vpos(s, q[0]), vpos(s, q[1]), vpos(s, q[2]), vpos(s, q[3]));
            } else {
                const int32_t* t = &s.triangles[3 * i];
                l.cdf[i] = triangle_area(vpos(s, t[0]), vpos(s, t[1]), vpos(s, t[2]));
            }
            if (i != 0) l.cdf[i] += l.cdf[i - 1];
        }
        lights.push_back(l);
    }
    const float pif = 3.14159265358979323846f;
    for (int32_t h = 0; h < scene->nenvironments; h++) {
        const jt_environment& e = scene->environments[h];
        if (e.emission[0] == 0 && e.emission[1] == 0 && e.emission[2] == 0) continue;
        if (e.emission_tex < 0 || e.emission_tex >= scene->ntextures) {
            cleanup();
            return fail(JT_ERR_UNSUPPORTED,
                        "emissive environment without texture: l_elements_cdf is undefined in the "
                        "reference (src/trace.jl:170-183)");
        }
        const jt_texture& t = scene->textures[e.emission_tex];
        jt_light l{-1, h, t.width * t.height, nullptr};
        l.cdf = (float*)std::malloc(sizeof(float) * std::max(1, l.ncdf));
        if (!l.cdf) {
            cleanup();
            return fail(JT_ERR_NOMEM, "out of host memory");
        }
        for (long idx = 0; idx < l.ncdf; idx++) {
            long i = idx % t.width, j = idx / t.width;
            float th = ((float)j + 0.5f) * pif / (float)t.height;
            long k = 4 * (j * (long)t.width + i);
            float v[4];
            for (int c = 0; c < 4; c++) v[c] = t.pixelsf ? t.pixelsf[k + c] : (float)t.pixelsb[k + c] / 255.0f;
            // maximum(value) over all four channels of lookup_texture(as_linear=false)
            float mv = jl_max(jl_max(jl_max(v[0], v[1]), v[2]), v[3]);
            l.cdf[idx] = mv * (float)std::sin((double)th);
            if (idx != 0) l.cdf[idx] += l.cdf[idx - 1];
        }
        lights.push_back(l);
    }
    out->nlights = (int32_t)lights.size();
    out->lights = (jt_light*)std::calloc(std::max<size_t>(1, lights.size()), sizeof(jt_light));
    if (!out->lights) {
        cleanup();
        return fail(JT_ERR_NOMEM, "out of host memory");
    }
    for (size_t k = 0; k < lights.size(); k++) out->lights[k] = lights[k];
    return JT_OK;
}

void jt_free_lights(jt_lights* lights) {
    if (!lights) return;
    if (lights->lights)
        for (int32_t i = 0; i < lights->nlights; i++) std::free(lights->lights[i].cdf);
    std::free(lights->lights);
    std::memset(lights, 0, sizeof(*lights));
}

// make_trace_state (src/trace.jl:189-197): longer side = resolution, other = round(res / aspect)
int jt_image_size(const jt_scene* scene, const jt_params* params, int32_t* width, int32_t* height) {
    if (!scene || !params || !width || !height) return fail(JT_ERR_INVALID, "NULL argument");
    if (params->width > 0 && params->height > 0) {
        *width = params->width;
        *height = params->height;
        return JT_OK;
    }
    if (params->camera < 0 || params->camera >= scene->ncameras)
        return fail(JT_ERR_INVALID, "camera id out of range");
    const float aspect = scene->cameras[params->camera].aspect;
    // Julia round(Int, x) rounds half to even; resolution / aspect is Int / Float32 -> Float32
    if (aspect >= 1) {
        *width = params->resolution;
        *height = (int32_t)std::nearbyint((float)params->resolution / aspect);
    } else {
        *height = params->resolution;
        *width = (int32_t)std::nearbyint((float)params->resolution * aspect);
    }
    if (*width <= 0 || *height <= 0) return fail(JT_ERR_INVALID, "empty image");
    return JT_OK;
}

}  // extern "C"
