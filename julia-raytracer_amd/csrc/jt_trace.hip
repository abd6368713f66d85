// jt_trace.hip — the C-ABI device context of the MI355X path tracer (include/jtrace.h): scene
// upload and layout, launches, the multi-device split and its RCCL reduce. The kernels are in
// jt_kernels.h (instantiated by jt_kv.hip, one translation unit per configuration).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "jt_internal.h"
#include "jt_kernels.h"

using namespace jtd;
using namespace jtk;

namespace jtk {
// every configuration is compiled in its own translation unit (jt_kv.hip)
JT_KV_FOR(0, extern template)
JT_KV_FOR(1, extern template)
JT_KV_FOR(2, extern template)
JT_KV_FOR(3, extern template)
JT_KV_FOR(4, extern template)
JT_KV_FOR(5, extern template)
JT_KV_FOR(6, extern template)
JT_KV_FOR(7, extern template)
JT_KV_FOR(8, extern template)
JT_KV_FOR(9, extern template)
JT_KV_FOR(10, extern template)
JT_KV_FOR(11, extern template)
JT_KV_FOR(12, extern template)
JT_KV_FOR(13, extern template)
JT_KV_FOR(14, extern template)
JT_KV_FOR(15, extern template)

// configuration ID of the binary traversal, or its wide twin (ID + NUM_BASE_CONFIGS)
template <int ID, int SAMPLER, int COUNT>
hipError_t launch_tw(bool wide, const DScene& S, const DParams& P, int s0, int s1, const DAccum& A, hipStream_t st, int cus) {
    return wide ? launch_cfg<ID + NUM_BASE_CONFIGS, SAMPLER, COUNT>(S, P, s0, s1, A, st, cus)
                : launch_cfg<ID, SAMPLER, COUNT>(S, P, s0, s1, A, st, cus);
}
// Stack configurations: the whole bound in a 16-entry LDS ring, or a RING-entry ring + HBM.
template <int SAMPLER, int COUNT>
hipError_t launch_s(int need, int ring, int kmask, bool wide, const DScene& S, const DParams& P, int s0, int s1,
                    const DAccum& A, hipStream_t st, int cus) {
    if (need <= 16) {
        if (kmask == (FT_NONE | FT_LINL)) return launch_tw<0, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
        if (kmask == FT_NONE) return launch_tw<7, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
        return launch_tw<1, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
    }
    if (ring <= 16) {
        switch (kmask) {
            case FT_MESH | FT_LINL: return launch_tw<2, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
            case FT_MESH_ENV | FT_NOIL: return launch_tw<3, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
            case FT_MESH_ENV_QUAD | FT_LINL: return launch_tw<4, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
            default: return launch_tw<5, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
        }
    }
    return launch_tw<6, SAMPLER, COUNT>(wide, S, P, s0, s1, A, st, cus);
}
}  // namespace jtk

// ============================================================================ C-ABI context
struct jt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    DScene S{};
    DParams P{};
    DAccum A{};
    std::vector<void*> allocations;
    int width = 0, height = 0;
    int total_samples = 0, batch = 1, sampler = 1;
    int cus = 256;   // compute units of the device (persistent grid size)
    int lk = 0;      // log2 of the sample streams per pixel (DParams::lk; fixed at jt_create)
    int tiles = 0;   // 8x8 pixel tiles
    int stack = 16;  // stack bound of the scene (entries); > 16: LDS ring of `ring` + HBM overflow
    int ring = 16;
    int feat = FT_ALL;   // scene feature bits (jt_device.h)
    int kmask = FT_ALL;  // feature mask of the kernel specialisation the scene runs
    bool wide = false;   // JT_TRAVERSAL_WIDE: the wide-record kernels (configurations 8-15)
    int traversal = 0;   // jt_params.traversal as resolved (JT_TRAVERSAL_AUTO: near or wide)
    int first = -1, next = 0;  // running-mean origin and next expected sample (deferred ones included)
    // Deferred samples [pend0, pend1): jt_trace_range / jt_trace_samples queue their range and
    // trace it, merged with the ranges queued before it, once JT_DEFER_SAMPLES are queued or when
    // anything reads the context (flush). A render split into calls gives the bits of one call
    // (jt_trace_range's contract), so merging changes only the launch count: the reference's
    // default --batch 1 (one call per sample) runs as launches of many samples each.
    int pend0 = 0, pend1 = 0;
    // one-stream contexts (lk == 0): a flushed range of m > 1 samples runs as chunks of up to
    // `chunk` samples, each traced as one-sample streams into the stream-mean buffers (allocated at
    // the first such flush) and folded into the running mean by chain_kernel in sample order
    int chunk = 0;
    // two sets of chunk buffers: chunk i traces into set i & 1 on `stream` while chain_kernel folds
    // chunk i - 1 on `stream2` (the chains stay in sample order on stream2; a trace reuses a set
    // only after the chain that read it, chain_done)
    float4* cpart[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
    hipStream_t stream2 = nullptr;
    hipEvent_t trace_done[2] = {nullptr, nullptr}, chain_done[2] = {nullptr, nullptr};
    bool exported = false;  // jt_get_device_buffers handed out the accumulators' device pointers
    int count = 1;             // 1: all traversal counters (diagnostic), 0: paths/rays/light queries only
    bool failed = false;       // a launch failed: the running means are unusable
    bool stale = true;         // the accumulators are not yet zeroed or overwritten since jt_reset
    // k > 1: the last launch combined the image only; albedo, normal and hits are combined from
    // the stream means (weights aov_cw) when first read (finish_aovs)
    bool aov_pending = false;
    DCombine aov_cw{};
    bool env_alias = false;    // JT_ENV_ALIAS=1: environment lights sample through alias tables
                               // until jt_reset
    size_t lds_scene_bytes = 0;  // > 0: small-scene LDS mode
    unsigned long long launches = 0;
    double kernel_ms = 0;
    // multi-device context (jt_create_multi): one sub-context per device, each tracing its share
    // of every batch into its own running mean; RCCL communicators for the reduce of jt_get_image
    std::vector<jt_ctx*> sub;
    std::vector<ncclComm_t> comms;
    std::vector<long long> nsub;  // samples accumulated by each device
    // split of every batch: false = contiguous sample shares (device d's mean weighted n_d / N in
    // the reduce), true = interleaved 8x8 pixel tiles (tile t on device t mod D, every sample of
    // the batch; disjoint pixels, so the reduce is a plain sum). Tiles when params.batch < D:
    // the reference's default --batch 1 would leave all but one device idle under a sample split
    bool tile_split = false;
    float* red = nullptr;         // device 0: reduce target, W*H float4
    long long* red_hits = nullptr;
};

namespace jtk {
// the combine of every pixel's stream means (DCombine, jt_kernels.h), one thread per pixel of
// the launch's tiles (slot g); stream j's records of neighbouring pixels are contiguous (coalesced).
// Two kernels over the same streams: the image after every launch (16 B per pixel and stream),
// the AOVs and hits (32 B per pixel and stream) only when they are read (jt_ctx::aov_pending):
// the stream means stay in place until the next launch appends to them, so the deferred AOV
// combine reads exactly what an eager one would have
template <bool AOV>
__global__ __launch_bounds__(256) void combine_kernel(DParams P, DAccum A, DCombine Cw) {
    const int tiles_x = (P.width + 7) / 8, tiles = launch_tiles(P);
    const int g = (int)(blockIdx.x * 256 + threadIdx.x);
    if (g >= tiles * 64) return;
    const int t = (g >> 6) * P.tile_stride + P.tile_offset, l = g & 63;
    const int i = (t % tiles_x) * 8 + (l & 7), j = (t / tiles_x) * 8 + (l >> 3);
    if (i >= P.width || j >= P.height) return;
    const size_t pixel = (size_t)j * P.width + i, ns = (size_t)A.nslot;
    const float w0 = Cw.w[0];
    if constexpr (!AOV) {
        float4 im = A.part_img[g];
        im = make_float4(im.x * w0, im.y * w0, im.z * w0, im.w * w0);
        // unrolled: eight streams' loads in flight per thread (the sums stay in stream order)
#pragma unroll 8
        for (int s = 1; s < Cw.ns; s++) {
            const float w = Cw.w[s];
            const float4 a = A.part_img[s * ns + g];
            im = make_float4(im.x + a.x * w, im.y + a.y * w, im.z + a.z * w, im.w + a.w * w);
        }
        A.image[pixel] = im;
    } else {
        float4 al = A.part_alb[g], nr = A.part_nrm[g];
        long long h = __float_as_int(al.w);
        al = make_float4(al.x * w0, al.y * w0, al.z * w0, 0.0f);
        nr = make_float4(nr.x * w0, nr.y * w0, nr.z * w0, 0.0f);
#pragma unroll 4
        for (int s = 1; s < Cw.ns; s++) {
            const float w = Cw.w[s];
            const float4 b = A.part_alb[s * ns + g], c = A.part_nrm[s * ns + g];
            al = make_float4(al.x + b.x * w, al.y + b.y * w, al.z + b.z * w, 0.0f);
            nr = make_float4(nr.x + c.x * w, nr.y + c.y * w, nr.z + c.z * w, 0.0f);
            h += __float_as_int(b.w);
        }
        A.albedo[pixel] = al;
        A.normal[pixel] = nr;
        A.hits[pixel] = h;
    }
}

// A chunk of a one-stream context (k = 1, the reference's single running mean): the chunk's
// samples x .. x+m-1 were traced as m one-sample streams (each record = that sample's value:
// 0 * 0 + value * 1), and are folded into the running mean here one by one, in sample order, with
// the epilogue's own operations (mean * (1 - w) + value * w, w = 1 / (n0 + j + 1): src/trace.jl:
// 631-648, src/math.jl:89-93) — bit for bit the image of tracing the samples one launch each.
// n0: the context's samples before the chunk (0: the mean starts from zero, as after jt_reset).
// At most 32 VGPRs: the trace kernel of the next chunk (5 waves/SIMD of 96 VGPRs in LDS mode)
// leaves 32 per SIMD free, so chain waves run on the same CUs beside it (stream2).
__global__ __launch_bounds__(256) void chain_kernel(DParams P, DAccum A, int n0, int m) {
    const int tiles_x = (P.width + 7) / 8, tiles = launch_tiles(P);
    const int g = (int)(blockIdx.x * 256 + threadIdx.x);
    if (g >= tiles * 64) return;
    const int t = (g >> 6) * P.tile_stride + P.tile_offset, l = g & 63;
    const int i = (t % tiles_x) * 8 + (l & 7), j = (t / tiles_x) * 8 + (l >> 3);
    if (i >= P.width || j >= P.height) return;
    const unsigned pixel = (unsigned)j * (unsigned)P.width + (unsigned)i;  // jt_create: < 2^26 pixels
    float ix = 0, iy = 0, iz = 0, iw = 0, ax = 0, ay = 0, az = 0, nx = 0, ny = 0, nz = 0;
    int h = 0;  // the chunk's hits (< 2^31 samples)
    if (n0 > 0) {
        const float4 a = A.image[pixel], b = A.albedo[pixel], c = A.normal[pixel];
        ix = a.x, iy = a.y, iz = a.z, iw = a.w, ax = b.x, ay = b.y, az = b.z, nx = c.x, ny = c.y, nz = c.z;
    }
    // few live registers (byte offsets below 4 GiB: 2^27 records of 16 B at most per buffer set
    // and array, jt_ctx::chunk), so the waves fit beside the next chunk's trace kernel
    const char* pi = reinterpret_cast<const char*>(A.part_img);
    const char* pa = reinterpret_cast<const char*>(A.part_alb);
    const char* pn = reinterpret_cast<const char*>(A.part_nrm);
    const unsigned step = (unsigned)A.nslot * 16u;
    unsigned off = (unsigned)g * 16u;
#pragma unroll 1
    for (int s = 0; s < m; s++, off += step) {
        const float w = 1.0f / (float)(n0 + s + 1), omw = 1 - w;
        const float4 a = *reinterpret_cast<const float4*>(pi + off);
        ix = ix * omw + a.x * w, iy = iy * omw + a.y * w, iz = iz * omw + a.z * w, iw = iw * omw + a.w * w;
        const float4 b = *reinterpret_cast<const float4*>(pa + off);
        ax = ax * omw + b.x * w, ay = ay * omw + b.y * w, az = az * omw + b.z * w;
        h += __float_as_int(b.w);
        const float4 c = *reinterpret_cast<const float4*>(pn + off);
        nx = nx * omw + c.x * w, ny = ny * omw + c.y * w, nz = nz * omw + c.z * w;
    }
    A.image[pixel] = make_float4(ix, iy, iz, iw);
    A.albedo[pixel] = make_float4(ax, ay, az, 0.0f);
    A.normal[pixel] = make_float4(nx, ny, nz, 0.0f);
    A.hits[pixel] = (n0 > 0 ? A.hits[pixel] : 0LL) + h;
}

}  // namespace jtk

namespace {

int hip_fail(hipError_t e, const char* what) {
    return jt::fail(JT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
int zero_if_stale(jt_ctx* c);

// RCCL, loaded on first use by a multi-device context (dlopen of the ROCm install's
// librccl.so.1): single-device contexts never touch it, and a process that already loaded an
// RCCL (e.g. torch's) shares that one instead of a second copy
struct Rccl {
    bool ok = false;
    decltype(&ncclCommInitAll) CommInitAll;
    decltype(&ncclCommDestroy) CommDestroy;
    decltype(&ncclReduce) Reduce;
    decltype(&ncclGroupStart) GroupStart;
    decltype(&ncclGroupEnd) GroupEnd;
    decltype(&ncclRedOpCreatePreMulSum) RedOpCreatePreMulSum;
    decltype(&ncclRedOpDestroy) RedOpDestroy;
    decltype(&ncclGetErrorString) GetErrorString;
};
const Rccl& rccl() {
    static Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return x;
        x.CommInitAll = (decltype(x.CommInitAll))dlsym(h, "ncclCommInitAll");
        x.CommDestroy = (decltype(x.CommDestroy))dlsym(h, "ncclCommDestroy");
        x.Reduce = (decltype(x.Reduce))dlsym(h, "ncclReduce");
        x.GroupStart = (decltype(x.GroupStart))dlsym(h, "ncclGroupStart");
        x.GroupEnd = (decltype(x.GroupEnd))dlsym(h, "ncclGroupEnd");
        x.RedOpCreatePreMulSum = (decltype(x.RedOpCreatePreMulSum))dlsym(h, "ncclRedOpCreatePreMulSum");
        x.RedOpDestroy = (decltype(x.RedOpDestroy))dlsym(h, "ncclRedOpDestroy");
        x.GetErrorString = (decltype(x.GetErrorString))dlsym(h, "ncclGetErrorString");
        x.ok = x.CommInitAll && x.CommDestroy && x.Reduce && x.GroupStart && x.GroupEnd && x.RedOpCreatePreMulSum &&
               x.RedOpDestroy && x.GetErrorString;
        return x;
    }();
    return r;
}
int nccl_fail(ncclResult_t r, const char* what) {
    return jt::fail(JT_ERR_DEVICE, std::string(what) + ": " + rccl().GetErrorString(r));
}

// Vose's alias table of the pmf a light CDF holds (p_i = cdf[i] - cdf[i-1], src/sampling.jl:39-40),
// appended to `out`: entry i = (probability of keeping column i, the other index of the column).
// Built in double; the JT_ENV_ALIAS variant's sample_lights reads it.
void build_alias_table(const float* cdf, int n, std::vector<float2>& out) {
    auto bits = [](int i) {
        float f;
        std::memcpy(&f, &i, 4);
        return f;
    };
    std::vector<double> q(n);
    double total = 0;
    for (int i = 0; i < n; i++) {
        q[i] = std::max(0.0, (double)cdf[i] - (i ? (double)cdf[i - 1] : 0.0));
        total += q[i];
    }
    const size_t base = out.size();
    out.resize(base + n);
    std::vector<int> small, large;
    for (int i = 0; i < n; i++) {
        q[i] = total > 0 ? q[i] * n / total : 1.0;
        (q[i] < 1.0 ? small : large).push_back(i);
    }
    while (!small.empty() && !large.empty()) {
        const int s = small.back(), l = large.back();
        small.pop_back();
        out[base + s] = make_float2((float)q[s], bits(l));
        q[l] -= 1.0 - q[s];
        if (q[l] < 1.0) {
            large.pop_back();
            small.push_back(l);
        }
    }
    for (int i : large) out[base + i] = make_float2(1.0f, bits(i));
    for (int i : small) out[base + i] = make_float2(1.0f, bits(i));  // rounding leftovers
}

template <class T>
int upload(jt_ctx* c, const std::vector<T>& host, const T** dptr) {
    size_t bytes = std::max<size_t>(sizeof(T), host.size() * sizeof(T));
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return jt::fail(JT_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    c->allocations.push_back(p);
    if (!host.empty()) {
        e = hipMemcpy(p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail(e, "hipMemcpy");
    }
    *dptr = (const T*)p;
    return JT_OK;
}

int tree_depth(const jt_bvh_tree& t) {
    if (t.nnodes == 0) return 0;
    std::vector<std::pair<int, int>> st{{0, 0}};
    int depth = 0;
    while (!st.empty()) {
        auto [n, d] = st.back();
        st.pop_back();
        depth = std::max(depth, d);
        const jt_bvh_node& nd = t.nodes[n];
        if (nd.internal) {
            st.push_back({nd.start, d + 1});
            st.push_back({nd.start + 1, d + 1});
        }
    }
    return depth;
}

inline float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }
inline float as_f(int v) {
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}
inline float as_f(unsigned v) {
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}
// the frame's x, y, z columns are bitwise the unit axes (+0 entries: a -0 could flip the sign
// of a zero normal component in transform_normal)
bool rot_identity(const float* fv) {
    const float id[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    return std::memcmp(fv, id, sizeof id) == 0;
}
DNode pack_node(const jt_bvh_node& n, int start) {
    unsigned meta = (unsigned)(uint16_t)n.num | ((unsigned)(uint8_t)n.axis << 16) | ((unsigned)(n.internal ? 1 : 0) << 24);
    return DNode{f4(n.bmin[0], n.bmax[0], n.bmin[1], n.bmax[1]), f4(n.bmin[2], n.bmax[2], as_f(start), as_f(meta))};
}

// ------------------------------------------------------------- wide records (JT_TRAVERSAL_WIDE)
// Conservative 8-bit quantisation of a child's slab [cmin, cmax] on one axis, relative to the
// record's origin o with scale s (a power of two): the largest lo with o + lo * s <= cmin and the
// smallest hi with o + hi * s >= cmax, evaluated in the device's float operations (wide_box,
// jt_kernels.h; -ffp-contract=off on both sides). false: no byte fits at this scale.
bool quantize_axis(float o, float s, float cmin, float cmax, unsigned& lo, unsigned& hi) {
    auto deq = [&](int q) { return o + (float)q * s; };
    int q = (int)std::max(0.0, std::min(255.0, std::floor(((double)cmin - (double)o) / (double)s)));
    while (q > 0 && deq(q) > cmin) q--;
    while (q < 255 && deq(q + 1) <= cmin) q++;
    if (!(deq(q) <= cmin)) return false;
    lo = (unsigned)q;
    q = (int)std::max(0.0, std::min(255.0, std::ceil(((double)cmax - (double)o) / (double)s)));
    while (q < 255 && deq(q) < cmax) q++;
    while (q > 0 && deq(q - 1) >= cmax) q--;
    if (!(deq(q) >= cmax)) return false;
    hi = (unsigned)q;
    return true;
}
float exp_scale(int e) {  // 2^(e - 127), e = a normal float's biased exponent
    const unsigned b = (unsigned)e << 23;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}
// The wide records of a binary tree: one per internal node N (or the root leaf), holding N's
// grandchildren in slots [LL, LR, RL, RR] (a leaf child takes the pair's first slot alone).
void wide_slots(const jt_bvh_tree& t, int n, int slot[4]) {
    slot[0] = slot[1] = slot[2] = slot[3] = -1;
    const jt_bvh_node& N = t.nodes[n];
    if (!N.internal) {
        slot[0] = n;
        return;
    }
    const int L = N.start, R = N.start + 1;
    if (t.nodes[L].internal) slot[0] = t.nodes[L].start, slot[1] = t.nodes[L].start + 1;
    else slot[0] = L;
    if (t.nodes[R].internal) slot[2] = t.nodes[R].start, slot[3] = t.nodes[R].start + 1;
    else slot[2] = R;
}
// Storage order of the wide records (the binary node each record stands for). JT_WIDE_ORDER 0:
// breadth-first. 1: sibling groups depth-first — a record's internal children are stored
// together, then each child's subtree in slot order, so a subtree is one contiguous run of
// records (a ray descending it stays in a few pages and L2 sets). Storage only: the traversal
// visits the same records in the same order. Measured against breadth-first (two runs each,
// profiles/r06_ab/wide_order_dfs_vs_bfs_r06d.txt): bathroom1 1920x1080x64 +0.1 %, ecosys
// 3840x2160x8 +0.2 %: within noise, so breadth-first stays the default.
#ifndef JT_WIDE_ORDER
#define JT_WIDE_ORDER 0
#endif
std::vector<int> wide_record_order(const jt_bvh_tree& t) {
    std::vector<int> seq;
    if (t.nnodes <= 0) return seq;
    seq.push_back(0);
    if (JT_WIDE_ORDER == 0) {
        for (size_t h = 0; h < seq.size(); h++) {
            if (!t.nodes[seq[h]].internal) continue;
            int slot[4];
            wide_slots(t, seq[h], slot);
            for (int c = 0; c < 4; c++)
                if (slot[c] >= 0 && t.nodes[slot[c]].internal) seq.push_back(slot[c]);
        }
        return seq;
    }
    // depth-first over sibling groups, iterative: a stack of the records whose children are still
    // to be appended (their subtrees then follow in slot order)
    std::vector<int> st{0};
    while (!st.empty()) {
        const int n = st.back();
        st.pop_back();
        if (!t.nodes[n].internal) continue;
        int slot[4];
        wide_slots(t, n, slot);
        int kids[4], nk = 0;
        for (int c = 0; c < 4; c++)
            if (slot[c] >= 0 && t.nodes[slot[c]].internal) kids[nk++] = slot[c];
        for (int c = 0; c < nk; c++) seq.push_back(kids[c]);
        for (int c = nk - 1; c >= 0; c--) st.push_back(kids[c]);
    }
    return seq;
}
// The binary leaves of a tree in the order the wide records list them: records in storage order
// (wide_record_order), within a record its leaf children in slot order. The device lays out
// primitive records and numbers instances in this order, so a record's leaf children are
// consecutive runs (a record could address them from one start) and every binary leaf is
// still one run (the binary traversal addresses a leaf by its start). Measured against node-index
// order: bathroom1 even, ecosys even (profiles/r05_ab/wide48_vs_wide64_r05f.txt "base"); it is
// what a record addressing its leaf children from one start needs (the 48-B record experiment,
// DESIGN.md §2).
std::vector<int> wide_leaf_order(const jt_bvh_tree& t) {
    std::vector<int> order;
    if (t.nnodes <= 0) return order;
    if (!t.nodes[0].internal) {
        order.push_back(0);
        return order;
    }
    for (int n : wide_record_order(t)) {
        int slot[4];
        wide_slots(t, n, slot);
        for (int c = 0; c < 4; c++)
            if (slot[c] >= 0 && !t.nodes[slot[c]].internal) order.push_back(slot[c]);
    }
    return order;
}

// The wide records of one binary tree, appended to `out` in wide_record_order (global indices =
// positions in `out`), their boxes quantised relative to N's box per axis at the smallest scale
// 2^(e-127) >= extent / 255 (and the next larger ones until every child fits). leaf_word(k): the
// child word of binary leaf k. Returns the root record's index, or -1 with the error set.
int build_wide(const jt_bvh_tree& t, const std::function<unsigned(int)>& leaf_word, std::vector<DWide>& out) {
    if (t.nnodes <= 0 || (!t.nodes[0].internal && t.nodes[0].num <= 0)) {
        // an empty tree (make_bvh of no boxes is one leaf without primitives, src/bvh.jl:138-183):
        // one record without children, so a query visits it and finds nothing
        DWide w{};
        w.r3 = make_uint4(W_EMPTY, W_EMPTY, W_EMPTY, W_EMPTY);
        out.push_back(w);
        return (int)out.size() - 1;
    }
    const std::vector<int> seq = wide_record_order(t);
    const size_t base = out.size();
    if (base + seq.size() > (size_t)IDX_MASK) return jt::fail(JT_ERR_UNSUPPORTED, "scene exceeds 2^24 wide records"), -1;
    std::vector<int> rec_of(t.nnodes, -1);  // binary internal node -> its record
    for (size_t h = 0; h < seq.size(); h++) rec_of[seq[h]] = (int)(base + h);
    out.resize(base + seq.size());
    for (size_t h = 0; h < seq.size(); h++) {
        const jt_bvh_node& N = t.nodes[seq[h]];
        int slot[4], a1 = 0, a2 = 0;
        wide_slots(t, seq[h], slot);
        if (N.internal) {
            if (t.nodes[N.start].internal) a1 = t.nodes[N.start].axis;
            if (t.nodes[N.start + 1].internal) a2 = t.nodes[N.start + 1].axis;
        }
        unsigned word[4] = {W_EMPTY, W_EMPTY, W_EMPTY, W_EMPTY};
        for (int c = 0; c < 4; c++) {
            if (slot[c] < 0) continue;
            const jt_bvh_node& C = t.nodes[slot[c]];
            if (C.internal) {
                word[c] = (unsigned)rec_of[slot[c]];
            } else {
                if (C.num < 1 || C.num > 4) return jt::fail(JT_ERR_UNSUPPORTED, "wide traversal: a BVH leaf outside 1..4 primitives"), -1;
                word[c] = leaf_word(slot[c]);
                if (word[c] == W_EMPTY) return -1;
            }
        }
        // quantisation per axis
        unsigned e3[3], lo[3][4] = {}, hi[3][4] = {};
        for (int ax = 0; ax < 3; ax++) {
            const float o = N.bmin[ax];
            bool finite = std::isfinite(N.bmin[ax]) && std::isfinite(N.bmax[ax]);
            for (int c = 0; c < 4; c++)
                if (slot[c] >= 0)
                    finite = finite && std::isfinite(t.nodes[slot[c]].bmin[ax]) && std::isfinite(t.nodes[slot[c]].bmax[ax]);
            if (!finite) return jt::fail(JT_ERR_UNSUPPORTED, "wide traversal: a non-finite BVH box"), -1;
            const double ext = (double)N.bmax[ax] - (double)N.bmin[ax];
            int e = 1;  // smallest biased exponent with 255 * 2^(e - 127) >= ext
            while (e < 254 && 255.0 * std::ldexp(1.0, e - 127) < ext) e++;
            for (;; e++) {
                if (e > 254) return jt::fail(JT_ERR_UNSUPPORTED, "wide traversal: a box cannot be quantised"), -1;
                const float sc = exp_scale(e);
                bool ok = std::isfinite(o + 255.0f * sc);
                for (int c = 0; c < 4 && ok; c++)
                    if (slot[c] >= 0)
                        ok = quantize_axis(o, sc, t.nodes[slot[c]].bmin[ax], t.nodes[slot[c]].bmax[ax], lo[ax][c], hi[ax][c]);
                if (ok) break;
            }
            e3[ax] = (unsigned)e;
        }
        auto bytes = [](const unsigned* v) { return v[0] | v[1] << 8 | v[2] << 16 | v[3] << 24; };
        DWide& W = out[base + h];
        const unsigned meta = e3[0] | e3[1] << 8 | e3[2] << 16 |
                              ((unsigned)(N.internal ? N.axis : 0) | (unsigned)a1 << 2 | (unsigned)a2 << 4) << 24;
        W.r0 = make_float4(N.bmin[0], N.bmin[1], N.bmin[2], as_f(meta));
        W.r1 = make_uint4(bytes(lo[0]), bytes(hi[0]), bytes(lo[1]), bytes(hi[1]));
        W.r2 = make_uint4(bytes(lo[2]), bytes(hi[2]), 0u, 0u);
        W.r3 = make_uint4(word[0], word[1], word[2], word[3]);
    }
    return (int)base;
}

// the launch schedule: a unit counter per XCD band
constexpr size_t SCHED_BYTES = (size_t)NBANDS * BAND_STRIDE * 4;

// Sample streams per pixel (DESIGN.md §2 "Sample streams"), fixed at jt_create from the pixels
// the context traces and the batch only (never from the scene's memory mode, so every option
// that picks LDS or HBM mode keeps the image bits): 1 for the reference's default one-sample
// batches (its single running mean); otherwise at least 16 — 32 from a batch of 64 (two samples
// per stream) — and enough for 2^22 (pixel, stream) items (a context tracing few pixels — a tile
// share, a small image — still fills the GPU), at most 64, the batch, and 2^27 items of stream
// means (6.4 GB).
// Measured (gpurun_out/r05i, r05j): bathroom1 1024 spp 8 -> 16 streams +0.8 %, features2 512 spp
// +2 %, ecosys 64 spp 2 -> 16 +2.6 %, its 1/8 share (512 spp) +3.7 %; a 1/8 tile share of the
// headline 32 streams 9265, 64 streams 9794 Mrays/s. A context whose scene runs from HBM starts
// from 32 streams when the batch gives each at least two samples (gpurun_out/r05sk, r05sk2:
// features2 +0.6 %, bathroom1 +0.5 %; cornellbox +1.0 %, round 5, when 32 streams were the
// HBM-mode rule only). The option "streams" overrides.
int stream_log2(long long pixels, int batch) {
    if (batch <= 1) return 0;
    long long want = batch >= 2 * JT_STREAMS_WIDE ? JT_STREAMS_WIDE : JT_STREAMS_MIN;
    while (pixels * want < JT_STREAM_ITEMS) want *= 2;
    int lk = 0;
    while (lk < 6 && (2LL << lk) <= want && (2 << lk) <= batch && (2 << lk) <= JT_MAX_STREAMS &&
           pixels * (2LL << lk) <= JT_STREAM_ITEMS_MAX)
        lk++;
    return lk;
}

int check_tree(const jt_bvh_tree& t, int nprims_expected, const char* what) {
    if (t.nprimitives != nprims_expected) return jt::fail(JT_ERR_INVALID, std::string(what) + ": primitive count mismatch");
    for (int k = 0; k < t.nnodes; k++) {
        const jt_bvh_node& n = t.nodes[k];
        if (n.internal) {
            if (n.start < 0 || n.start + 1 >= t.nnodes) return jt::fail(JT_ERR_INVALID, std::string(what) + ": bad child index");
        } else if (n.start < 0 || n.num < 0 || n.start + n.num > t.nprimitives) {
            return jt::fail(JT_ERR_INVALID, std::string(what) + ": bad leaf range");
        } else if (n.num > 4) {  // make_bvh's leaves hold at most BVH_MAX_PRIMS (src/bvh.jl:32,166)
            return jt::fail(JT_ERR_INVALID, std::string(what) + ": a leaf above BVH_MAX_PRIMS (4) primitives");
        }
    }
    for (int k = 0; k < t.nprimitives; k++)
        if (t.primitives[k] < 0 || t.primitives[k] >= nprims_expected)
            return jt::fail(JT_ERR_INVALID, std::string(what) + ": bad primitive id");
    return JT_OK;
}

// srgb_to_rgb(byte_to_float(b)) (src/color.jl:12-23), the power evaluated in double
void build_luts(std::vector<float>& srgb, std::vector<float>& bytes) {
    srgb.resize(256);
    bytes.resize(256);
    for (int b = 0; b < 256; b++) {
        float c = (float)b / 255.0f;
        bytes[b] = c;
        srgb[b] = c <= 0.04045f ? c / 12.92f : (float)std::pow((double)((c + 0.055f) / 1.055f), (double)2.4f);
    }
}

}  // namespace

extern "C" {

int jt_device_count(int32_t* out) {
    if (!out) return jt::fail(JT_ERR_INVALID, "out is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *out = 0;
        return hip_fail(e, "hipGetDeviceCount");
    }
    *out = n;
    return JT_OK;
}

void jt_destroy(jt_ctx* c) {
    if (!c) return;
    if (!c->sub.empty() || !c->comms.empty()) {
        for (ncclComm_t m : c->comms) (void)rccl().CommDestroy(m);
        if (!c->sub.empty()) {
            (void)hipSetDevice(c->sub[0]->device);
            if (c->red) (void)hipFree(c->red);
            if (c->red_hits) (void)hipFree(c->red_hits);
        }
        for (jt_ctx* s : c->sub) jt_destroy(s);
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->stream2) (void)hipStreamSynchronize(c->stream2);
    for (void* p : c->allocations) (void)hipFree(p);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (int k = 0; k < 2; k++) {
        if (c->trace_done[k]) (void)hipEventDestroy(c->trace_done[k]);
        if (c->chain_done[k]) (void)hipEventDestroy(c->chain_done[k]);
    }
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int jt_create(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights, const jt_params* params,
              jt_ctx** out) {
    if (!out) return jt::fail(JT_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (!scene || !bvh || !lights || !params) return jt::fail(JT_ERR_INVALID, "NULL argument");
    if (params->camera < 0 || params->camera >= scene->ncameras) return jt::fail(JT_ERR_INVALID, "camera id out of range");
    if (params->sampler != JT_SAMPLER_PATH && params->sampler != JT_SAMPLER_NAIVE)
        return jt::fail(JT_ERR_INVALID, "sampler must be 1 (path) or 2 (naive)");
    if (params->samples < 0 || params->bounces < 0 || params->batch < 1)
        return jt::fail(JT_ERR_INVALID, "samples/bounces must be >= 0 and batch >= 1");
    if (params->bounces > 32766)  // the kernel keeps bounce in 15 bits of the path's control word
        return jt::fail(JT_ERR_UNSUPPORTED, "bounces above 32766 are not supported");
    if (bvh->nshapes != scene->nshapes) return jt::fail(JT_ERR_INVALID, "bvh.nshapes != scene.nshapes");
    // ------------------------------------------------------------- validate what the reference can shade
    for (int s = 0; s < scene->nshapes; s++) {
        const jt_shape& sh = scene->shapes[s];
        if (sh.npoints > 0 || (sh.nlines > 0 && sh.ntriangles == 0 && sh.nquads == 0))
            return jt::fail(JT_ERR_UNSUPPORTED, "shape " + std::to_string(s) +
                                                    ": points/lines are not shaded by the reference (src/scene.jl:429,605)");
        if (sh.ntriangles == 0 && sh.nquads == 0)
            return jt::fail(JT_ERR_UNSUPPORTED, "shape " + std::to_string(s) + " has no triangles or quads");
        if (sh.nnormals != 0 && sh.nnormals != sh.npositions)
            return jt::fail(JT_ERR_INVALID, "shape " + std::to_string(s) + ": normals/positions length mismatch");
        if (sh.ntexcoords != 0 && sh.ntexcoords != sh.npositions)
            return jt::fail(JT_ERR_INVALID, "shape " + std::to_string(s) + ": texcoords/positions length mismatch");
        if (sh.ncolors != 0 && sh.ncolors != sh.npositions)
            return jt::fail(JT_ERR_INVALID, "shape " + std::to_string(s) + ": colors/positions length mismatch");
        const int32_t* idx = sh.ntriangles ? sh.triangles : sh.quads;
        long n = sh.ntriangles ? 3L * sh.ntriangles : 4L * sh.nquads;
        for (long k = 0; k < n; k++)
            if (idx[k] < 0 || idx[k] >= sh.npositions)
                return jt::fail(JT_ERR_INVALID, "shape " + std::to_string(s) + ": vertex id out of range");
    }
    for (int k = 0; k < scene->ninstances; k++) {
        const jt_instance& in = scene->instances[k];
        if (in.shape < 0 || in.shape >= scene->nshapes || in.material < 0 || in.material >= scene->nmaterials)
            return jt::fail(JT_ERR_INVALID, "instance " + std::to_string(k) + ": invalid shape/material id");
        if (scene->materials[in.material].type == JT_GLTFPBR)
            return jt::fail(JT_ERR_UNSUPPORTED, "instance " + std::to_string(k) +
                                                    ": gltfpbr calls undefined functions in the reference (src/shading.jl:254-321)");
    }
    auto tex_ok = [&](int t) { return t >= -1 && t < scene->ntextures; };
    for (int k = 0; k < scene->nmaterials; k++) {
        const jt_material& m = scene->materials[k];
        if (m.type < 0 || m.type > JT_GLTFPBR) return jt::fail(JT_ERR_INVALID, "material type out of range");
        if (!tex_ok(m.emission_tex) || !tex_ok(m.color_tex) || !tex_ok(m.roughness_tex) || !tex_ok(m.scattering_tex) ||
            !tex_ok(m.normal_tex))
            return jt::fail(JT_ERR_INVALID, "material " + std::to_string(k) + ": texture id out of range");
    }
    for (int k = 0; k < scene->nenvironments; k++)
        if (!tex_ok(scene->environments[k].emission_tex)) return jt::fail(JT_ERR_INVALID, "environment texture id out of range");
    for (int k = 0; k < lights->nlights; k++) {
        const jt_light& l = lights->lights[k];
        if ((l.instance >= 0) == (l.environment >= 0) || l.ncdf <= 0 || !l.cdf)
            return jt::fail(JT_ERR_INVALID, "light " + std::to_string(k) + ": malformed");
        if (l.instance >= scene->ninstances || l.environment >= scene->nenvironments)
            return jt::fail(JT_ERR_INVALID, "light " + std::to_string(k) + ": id out of range");
        if (l.environment >= 0 && scene->environments[l.environment].emission_tex < 0)
            return jt::fail(JT_ERR_UNSUPPORTED, "untextured environment light: sample_sphere is undefined (src/trace.jl:1003)");
    }
    int st = check_tree(bvh->tlas, scene->ninstances, "tlas");
    if (st != JT_OK) return st;
    // the device numbers instances by TLAS leaf, leaves in wide-record order (wide_leaf_order), a
    // leaf's instances in its own order: a leaf's instances are then the id range start ..
    // start+num-1 (no per-instance index load) and a wide record's leaf children one range. The
    // TLAS must list each instance once.
    std::vector<int> inst_new(scene->ninstances, -1);  // reference instance id -> device id
    std::vector<int> tleaf_start(std::max(0, bvh->tlas.nnodes), 0);  // binary TLAS leaf -> first device id
    {
        int next = 0;
        for (int k : wide_leaf_order(bvh->tlas)) {
            const jt_bvh_node& n = bvh->tlas.nodes[k];
            tleaf_start[k] = next;
            for (int q = 0; q < n.num; q++) {
                int& slot = inst_new[bvh->tlas.primitives[n.start + q]];
                if (slot >= 0) return jt::fail(JT_ERR_INVALID, "tlas: an instance is listed twice");
                slot = next++;
            }
        }
        for (int& v : inst_new)  // instances no TLAS leaf lists are never visited
            if (v < 0) v = next++;
    }
    if (st != JT_OK) return st;
    int max_blas_depth = 0;
    for (int s = 0; s < scene->nshapes; s++) {
        const jt_shape& sh = scene->shapes[s];
        st = check_tree(bvh->blas[s], sh.ntriangles ? sh.ntriangles : sh.nquads, "blas");
        if (st != JT_OK) return st;
        max_blas_depth = std::max(max_blas_depth, tree_depth(bvh->blas[s]));
    }
    const int tlas_depth = tree_depth(bvh->tlas);
    // the reference's stacks hold bvhstacksize entries each; a DFS needs depth + 1
    if (std::max(tlas_depth, max_blas_depth) + 1 > params->bvhstacksize)
        return jt::fail(JT_ERR_STACK, "BVH deeper than --bvhstacksize (the reference throws BoundsError)");
    const int need = tlas_depth + max_blas_depth + 6;  // unified stack bound

    // the run-time options (jt_set_option) this context is created with
    const std::map<std::string, std::string> opts = jt::options_snapshot();
    auto opt = [&](const char* k) -> const char* {
        const auto it = opts.find(k);
        return it == opts.end() ? nullptr : it->second.c_str();
    };
    int32_t W = 0, H = 0;
    st = jt_image_size(scene, params, &W, &H);
    if (st != JT_OK) return st;

    hipError_t e = hipSetDevice(params->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    jt_ctx* c = new jt_ctx();
    c->device = params->device;
    c->width = W;
    c->height = H;
    c->total_samples = params->samples;
    c->batch = params->batch;
    c->sampler = params->sampler;
    c->stack = need;
    {  // scene feature bits (jt_device.h): scenes with none of them run the FT_NONE kernel
        int f = scene->nenvironments > 0 ? FT_ENV : 0;
        for (int k = 0; k < scene->nmaterials; k++) {
            const jt_material& m = scene->materials[k];
            if (m.type != JT_MATTE) f |= FT_MAT;
            if (m.type == JT_REFRACTIVE || m.type == JT_VOLUMETRIC || m.type == JT_SUBSURFACE) f |= FT_VOL;
            if (m.emission_tex >= 0 || m.color_tex >= 0 || m.roughness_tex >= 0 || m.scattering_tex >= 0 ||
                m.normal_tex >= 0)
                f |= FT_TEX;
            // opacity = m.opacity * color_tex.w * color_shp.w (src/scene.jl:649): a bilinear or
            // barycentric alpha of 1s need not round to exactly 1, so any color texture counts
            if (m.opacity < 1 || m.color_tex >= 0) f |= FT_OPAC;
        }
        for (int k = 0; k < scene->nshapes; k++) {
            const jt_shape& sh = scene->shapes[k];
            if (sh.nquads > 0) f |= FT_QUAD;
            if (sh.nnormals > 0 || sh.ntexcoords > 0 || sh.ncolors > 0) f |= FT_ATTR;
            if (sh.ncolors > 0) f |= FT_OPAC;
        }
        const char* fe = opt("features");
        c->feat = (fe && std::strcmp(fe, "all") == 0) ? FT_ALL : f;
    }
    if (const char* r = opt("lds_stack")) c->ring = std::atoi(r) > 16 ? 32 : 16;
    auto bail = [&](int status) {
        jt_destroy(c);
        return status;
    };
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return bail(hip_fail(e, "hipStreamCreate"));
    if ((e = hipEventCreate(&c->ev0)) != hipSuccess || (e = hipEventCreate(&c->ev1)) != hipSuccess)
        return bail(hip_fail(e, "hipEventCreate"));

    // ------------------------------------------------------------- flatten to the HBM layout
    // The TLAS is stored breadth-first (sibling pairs stay adjacent, the root stays node 0), so its
    // top levels share cache lines. Storage order only: the traversal still visits the
    // reference's nodes in the reference's order.
    std::vector<DNode> tlas;
    {
        const int tn = std::max(0, bvh->tlas.nnodes);
        std::vector<int> order, newidx(tn, -1);
        if (tn > 0) order.push_back(0);
        for (size_t q = 0; q < order.size(); q++) {
            const jt_bvh_node& n = bvh->tlas.nodes[order[q]];
            if (n.internal) {
                order.push_back(n.start);
                order.push_back(n.start + 1);
            }
        }
        for (size_t q = 0; q < order.size(); q++) newidx[order[q]] = (int)q;
        tlas.resize(order.size());
        for (size_t q = 0; q < order.size(); q++) {
            const jt_bvh_node& n = bvh->tlas.nodes[order[q]];
            tlas[q] = pack_node(n, n.internal ? newidx[n.start] : tleaf_start[order[q]]);
        }
    }
    std::vector<DNode> blas;
    std::vector<float4> prims;
    std::vector<DShape> shapes(scene->nshapes);
    std::vector<float4> pos, nrm, col;
    std::vector<float2> tc;
    std::vector<int4> elems;
    std::vector<float4> enrm, enrm_id;
    // the record (pair / quad) where each binary BLAS leaf's primitives start: the wide records'
    // leaf words (JT_TRAVERSAL_WIDE)
    std::vector<std::vector<int>> leaf_rec(scene->nshapes);
    for (int s = 0; s < scene->nshapes; s++) {
        const jt_shape& sh = scene->shapes[s];
        const jt_bvh_tree& t = bvh->blas[s];
        DShape& d = shapes[s];
        d.kind = sh.ntriangles ? KIND_TRI : KIND_QUAD;
        const int stride = d.kind == KIND_TRI ? 5 : 4;
        d.blas_root = (int)tlas.size() + (int)blas.size();  // global index: TLAS nodes come first
        // records are triangle pairs of 5 float4s or quads of 4: align the shape's first record to
        // its stride so prim_base * stride addresses it exactly when shape kinds are mixed
        while (prims.size() % stride) prims.push_back(f4(0, 0, 0, 0));
        d.prim_base = (int)(prims.size() / stride);  // in records
        d.idx_base = (int)elems.size();
        d.pos_base = (int)pos.size();
        for (int v = 0; v < sh.npositions; v++) pos.push_back(f4(sh.positions[3 * v], sh.positions[3 * v + 1], sh.positions[3 * v + 2], 0));
        d.nrm_base = -1;
        d.tc_base = -1;
        d.col_base = -1;
        // per-vertex attribute arrays are padded to the positions' base so one vertex id serves all
        if (sh.nnormals) {
            while ((int)nrm.size() < d.pos_base) nrm.push_back(f4(0, 0, 0, 0));
            d.nrm_base = (int)nrm.size();
            for (int v = 0; v < sh.nnormals; v++) nrm.push_back(f4(sh.normals[3 * v], sh.normals[3 * v + 1], sh.normals[3 * v + 2], 0));
        }
        if (sh.ntexcoords) {
            while ((int)tc.size() < d.pos_base) tc.push_back(make_float2(0, 0));
            d.tc_base = (int)tc.size();
            for (int v = 0; v < sh.ntexcoords; v++) tc.push_back(make_float2(sh.texcoords[2 * v], sh.texcoords[2 * v + 1]));
        }
        if (sh.ncolors) {
            while ((int)col.size() < d.pos_base) col.push_back(f4(0, 0, 0, 0));
            d.col_base = (int)col.size();
            for (int v = 0; v < sh.ncolors; v++)
                col.push_back(f4(sh.colors[4 * v], sh.colors[4 * v + 1], sh.colors[4 * v + 2], sh.colors[4 * v + 3]));
        }
        const int nel = d.kind == KIND_TRI ? sh.ntriangles : sh.nquads;
        leaf_rec[s].assign(t.nnodes, -1);
        // element normals (triangle_normal / quad_normal, src/geometry.jl:260-271) and their
        // transform_normal by an unrotated frame: host float ops identical to the device's
        for (int k = 0; k < nel; k++) {
            const int* v = d.kind == KIND_TRI ? &sh.triangles[3 * k] : &sh.quads[4 * k];
            auto P3 = [&](int vi) { return jt::mk3(sh.positions[3 * vi], sh.positions[3 * vi + 1], sh.positions[3 * vi + 2]); };
            auto tri_n = [](jt::f3 a, jt::f3 b, jt::f3 cc) { return jt::normalize(jt::cross(b - a, cc - a)); };
            jt::f3 n = d.kind == KIND_TRI ? tri_n(P3(v[0]), P3(v[1]), P3(v[2]))
                                          : jt::normalize(tri_n(P3(v[0]), P3(v[1]), P3(v[3])) + tri_n(P3(v[2]), P3(v[3]), P3(v[1])));
            const jt::frame3 I{jt::mk3(1, 0, 0), jt::mk3(0, 1, 0), jt::mk3(0, 0, 1), jt::mk3(0, 0, 0)};
            const jt::f3 ni = jt::normalize(jt::transform_vector(I, n));
            enrm.push_back(f4(n.x, n.y, n.z, 0));
            enrm_id.push_back(f4(ni.x, ni.y, ni.z, 0));
        }
        for (int k = 0; k < nel; k++) {
            if (d.kind == KIND_TRI)
                elems.push_back(make_int4(d.pos_base + sh.triangles[3 * k], d.pos_base + sh.triangles[3 * k + 1],
                                          d.pos_base + sh.triangles[3 * k + 2], 0));
            else
                elems.push_back(make_int4(d.pos_base + sh.quads[4 * k], d.pos_base + sh.quads[4 * k + 1],
                                          d.pos_base + sh.quads[4 * k + 2], d.pos_base + sh.quads[4 * k + 3]));
        }
        auto P3 = [&](int vi) { return f4(sh.positions[3 * vi], sh.positions[3 * vi + 1], sh.positions[3 * vi + 2], 0); };
        // records leaf by leaf, the leaves in wide-record order (wide_leaf_order: a wide record's
        // leaf children are consecutive runs); a leaf's records are its primitives in the
        // reference's order (bvh.primitives[start .. start+num-1]), pre-gathered
        const std::vector<int> lorder = wide_leaf_order(t);
        {
            int at = 0;
            for (int k : lorder) {
                leaf_rec[s][k] = d.prim_base + at;
                at += d.kind == KIND_TRI ? (t.nodes[k].num + 1) / 2 : t.nodes[k].num;
            }
        }
        for (int k = 0; k < t.nnodes; k++) {
            const jt_bvh_node& n = t.nodes[k];
            blas.push_back(pack_node(n, n.internal ? d.blas_root + n.start : std::max(0, leaf_rec[s][k])));
        }
        for (int k : lorder) {
            const jt_bvh_node& n = t.nodes[k];
            if (d.kind == KIND_TRI) {
                // Triangle-pair records (a leaf starts a record; an odd leaf's last record has a
                // zero second triangle, never accepted: the leaf count masks it). The two
                // triangles' components are interleaved so the pair test runs on packed FP32:
                //   (p1x p1x' p1y p1y') (p1z p1z' e1x e1x') (e1y e1y' e1z e1z') (e2x e2x' e2y e2y')
                //   (e2z e2z' el el'), edge1 = p2 - p1, edge2 = p3 - p1 (src/geometry.jl:208-209).
                for (int q = 0; q < n.num; q += 2) {
                    float4 p[2], e1[2], e2[2];
                    int el[2] = {-1, -1};
                    for (int h = 0; h < 2; h++) {
                        p[h] = e1[h] = e2[h] = f4(0, 0, 0, 0);
                        if (q + h >= n.num) continue;
                        el[h] = t.primitives[n.start + q + h];
                        const int* v = &sh.triangles[3 * el[h]];
                        const float4 a = P3(v[0]), b = P3(v[1]), cc = P3(v[2]);
                        p[h] = a;
                        e1[h] = f4(b.x - a.x, b.y - a.y, b.z - a.z, 0);
                        e2[h] = f4(cc.x - a.x, cc.y - a.y, cc.z - a.z, 0);
                    }
                    prims.push_back(f4(p[0].x, p[1].x, p[0].y, p[1].y));
                    prims.push_back(f4(p[0].z, p[1].z, e1[0].x, e1[1].x));
                    prims.push_back(f4(e1[0].y, e1[1].y, e1[0].z, e1[1].z));
                    prims.push_back(f4(e2[0].x, e2[1].x, e2[0].y, e2[1].y));
                    prims.push_back(f4(e2[0].z, e2[1].z, as_f(el[0]), as_f(el[1])));
                }
            } else {
                // quad records (the reference reads positions through bvh.primitives[i])
                for (int q = 0; q < n.num; q++) {
                    const int el = t.primitives[n.start + q];
                    const int* v = &sh.quads[4 * el];
                    float4 a = P3(v[0]), b = P3(v[1]), cc = P3(v[2]), dd = P3(v[3]);
                    a.w = as_f(el);
                    const bool degenerate = cc.x == dd.x && cc.y == dd.y && cc.z == dd.z;  // p3 == p4
                    dd.w = degenerate ? 1.0f : 0.0f;
                    prims.push_back(a);
                    prims.push_back(b);
                    prims.push_back(cc);
                    prims.push_back(dd);
                }
            }
        }
    }
    // wide records (JT_TRAVERSAL_WIDE): the TLAS's, then every BLAS's; the binary node array is
    // then not uploaded. JT_TRAVERSAL_AUTO resolves to near for a small scene that runs from LDS
    // or a shallow one, and to wide otherwise (decided with the LDS blob below; the records are
    // built then).
    if (params->traversal < JT_TRAVERSAL_REFERENCE || params->traversal > JT_TRAVERSAL_AUTO)
        return bail(jt::fail(JT_ERR_INVALID, "traversal must be 0 (reference), 1 (near), 2 (wide) or 3 (auto)"));
    c->wide = params->traversal == JT_TRAVERSAL_WIDE;
    std::vector<DWide> wnodes;
    std::vector<int> wroot(scene->nshapes, 0);
    int tlas_wnodes = 0;
    auto build_all_wide = [&]() -> int {
        const int r = build_wide(bvh->tlas, [&](int k) -> unsigned {
            const jt_bvh_node& n = bvh->tlas.nodes[k];
            return W_LEAF | W_INST | (unsigned)(n.num - 1) << 28 | (unsigned)tleaf_start[k];
        }, wnodes);
        if (r < 0) return JT_ERR_UNSUPPORTED;
        tlas_wnodes = (int)wnodes.size();
        for (int s = 0; s < scene->nshapes; s++) {
            const jt_bvh_tree& t = bvh->blas[s];
            wroot[s] = build_wide(t, [&](int k) -> unsigned {
                const int st0 = leaf_rec[s][k];
                if (st0 < 0 || st0 > (int)IDX_MASK) return jt::fail(JT_ERR_UNSUPPORTED, "wide traversal: too many primitive records"), (unsigned)W_EMPTY;
                return W_LEAF | (unsigned)(t.nodes[k].num - 1) << 28 | (unsigned)st0;
            }, wnodes);
            if (wroot[s] < 0) return JT_ERR_UNSUPPORTED;
        }
        return JT_OK;
    };
    if (c->wide && (st = build_all_wide()) != JT_OK) return bail(st);
    std::vector<DInstTrav> itrav(scene->ninstances);
    std::vector<int4> iblas(scene->ninstances);
    std::vector<DInstShade> ishade(scene->ninstances);
    for (int k0 = 0; k0 < scene->ninstances; k0++) {  // k0: the reference's id, k: the device's
        const int k = inst_new[k0];
        const jt_instance& in = scene->instances[k0];
        jt::frame3 f = jt::load_frame(in.frame);
        jt::frame3 inv = jt::inverse_frame(f, true);
        float iv[12], fv[12];
        jt::store_frame(inv, iv);
        jt::store_frame(f, fv);
        const DShape& d = shapes[in.shape];
        itrav[k] = DInstTrav{f4(iv[0], iv[1], iv[2], iv[3]), f4(iv[4], iv[5], iv[6], iv[7]), f4(iv[8], iv[9], iv[10], iv[11]),
                             in.shape, d.blas_root, d.kind, d.prim_base};
        // identity inverse (exact 1/0 entries, zero offset): transform_ray is the identity on
        // floats, so the traversal reuses the world ray (bit-identical)
        const float idm[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0};
        bool ident = true;
        for (int q = 0; q < 12; q++) ident = ident && iv[q] == idm[q];
        // jtk::node_step reads x, y (z); the wide traversal's x is the BLAS's root record; y the
        // identity inverse; w the shape, with bit 30 (jtk::INST_LEAF_ROOT) set for a one-leaf BLAS:
        // its intersect_instance_bvh tests the leaf's primitives in order whatever the child order,
        // so an exact-t tie there needs no re-run in the reference's order (jtk::rerun_tie)
        const jt_bvh_tree& bt = bvh->blas[in.shape];
        const bool leaf_root = bt.nnodes > 0 && !bt.nodes[0].internal;
        iblas[k] = make_int4(c->wide ? wroot[in.shape] : d.blas_root, ident ? 1 : 0, d.kind, in.shape | (leaf_root ? 1 << 30 : 0));
        if (!ident) c->feat |= FT_XFORM;
        ishade[k] = DInstShade{f4(fv[0], fv[1], fv[2], fv[3]), f4(fv[4], fv[5], fv[6], fv[7]), f4(fv[8], fv[9], fv[10], fv[11]),
                               in.material, in.shape, scene->materials[in.material].type,
                               rot_identity(fv) ? 1 : 0};
    }
    std::vector<DMaterial> mats(scene->nmaterials);
    for (int k = 0; k < scene->nmaterials; k++) {
        const jt_material& m = scene->materials[k];
        DMaterial& d = mats[k];
        std::memset(&d, 0, sizeof(d));
        d.type = m.type;
        d.emission_tex = m.emission_tex;
        d.color_tex = m.color_tex;
        d.roughness_tex = m.roughness_tex;
        d.scattering_tex = m.scattering_tex;
        d.normal_tex = m.normal_tex;
        for (int q = 0; q < 3; q++) {
            d.emission[q] = m.emission[q];
            d.color[q] = m.color[q];
            d.scattering[q] = m.scattering[q];
        }
        d.roughness = m.roughness;
        d.metallic = m.metallic;
        d.ior = m.ior;
        d.scanisotropy = m.scanisotropy;
        d.trdepth = m.trdepth;
        d.opacity = m.opacity;
    }
    std::vector<DTexture> texs(scene->ntextures);
    std::vector<uchar4> texb;
    std::vector<float4> texf;
    for (int k = 0; k < scene->ntextures; k++) {
        const jt_texture& t = scene->textures[k];
        DTexture& d = texs[k];
        std::memset(&d, 0, sizeof(d));
        d.width = t.width;
        d.height = t.height;
        d.linear = t.linear;
        d.is_float = t.pixelsf != nullptr;
        const size_t n = (size_t)t.width * (size_t)t.height;
        if (d.is_float) {
            d.offset = (long long)texf.size();
            for (size_t q = 0; q < n; q++)
                texf.push_back(f4(t.pixelsf[4 * q], t.pixelsf[4 * q + 1], t.pixelsf[4 * q + 2], t.pixelsf[4 * q + 3]));
        } else {
            if (!t.pixelsb && n) return bail(jt::fail(JT_ERR_INVALID, "texture without pixels"));
            d.offset = (long long)texb.size();
            for (size_t q = 0; q < n; q++)
                texb.push_back(make_uchar4(t.pixelsb[4 * q], t.pixelsb[4 * q + 1], t.pixelsb[4 * q + 2], t.pixelsb[4 * q + 3]));
        }
    }
    // one padding texel: eval_texture loads texels (i, j) and (i + 1, j) as one 8-B pair, which
    // past a texture's last texel reads one texel beyond it (and ignores it)
    texb.push_back(make_uchar4(0, 0, 0, 0));
    std::vector<DEnv> envs(scene->nenvironments);
    for (int k = 0; k < scene->nenvironments; k++) {
        const jt_environment& en = scene->environments[k];
        DEnv& d = envs[k];
        std::memset(&d, 0, sizeof(d));
        jt::frame3 f = jt::load_frame(en.frame);
        jt::store_frame(f, d.frame);
        jt::store_frame(jt::inverse_frame(f, false), d.inv);
        for (int q = 0; q < 3; q++) d.emission[q] = en.emission[q];
        d.tex = en.emission_tex;
    }
    std::vector<DLight> dl(lights->nlights);
    std::vector<float> cdf, guide_t;
    std::vector<int> guide_a;
    std::vector<float2> alias;
    const char* ea = opt("env_alias");
    const bool env_alias = ea && std::atoi(ea) != 0;
    c->env_alias = env_alias;
    for (int k = 0; k < lights->nlights; k++) {
        const jt_light& l = lights->lights[k];
        dl[k] = DLight{l.instance >= 0 ? inst_new[l.instance] : -1, l.environment, (int)cdf.size(), l.ncdf, 0, 0, 0.0f, -1};
        cdf.insert(cdf.end(), l.cdf, l.cdf + l.ncdf);
        const float last = l.ncdf > 0 ? l.cdf[l.ncdf - 1] : 0.0f;
        bool monotone = true;
        for (int i = 1; i < l.ncdf && monotone; i++) monotone = l.cdf[i] >= l.cdf[i - 1];
        if (l.ncdf >= 1024 && monotone && last > 0 && std::isfinite(last)) {
            // K buckets of the value range; K + 1 thresholds, the last one = last(cdf)
            const int K = std::min(65536, l.ncdf / 16);
            dl[k].guide_offset = (int)guide_t.size();
            dl[k].nguide = K;
            dl[k].guide_scale = (float)K / last;
            for (int b = 0; b <= K; b++) {
                const float t = b == K ? last : (float)((double)last * b / K);
                // first index with cdf[i] > t (n if none)
                const int a = (int)(std::upper_bound(l.cdf, l.cdf + l.ncdf, t) - l.cdf);
                guide_t.push_back(t);
                guide_a.push_back(a);
            }
            if (env_alias && l.environment >= 0) {
                dl[k].alias_offset = (int)alias.size();
                build_alias_table(l.cdf, l.ncdf, alias);
            }
        }
    }
    // light-hit records (DLightElem, jt_device.h): per instance light, one per element of its shape
    std::vector<int4> lhit(std::max(1, lights->nlights), make_int4(-1, 0, 0, 0));
    std::vector<float4> lelems;
    for (int k = 0; k < lights->nlights; k++) {
        const int inst = dl[k].instance;
        if (inst < 0) continue;
        const DInstShade& is = ishade[inst];
        const DShape& d = shapes[is.shape];
        const jt_shape& sh = scene->shapes[is.shape];
        const int nel = d.kind == KIND_TRI ? sh.ntriangles : sh.nquads;
        const float area = lights->lights[k].ncdf > 0 ? lights->lights[k].cdf[lights->lights[k].ncdf - 1] : 0.0f;
        lhit[k] = make_int4(inst, (int)(lelems.size() / 5), 0, 0);
        for (int e = 0; e < nel; e++) {
            const int g = d.idx_base + e;
            const int4 v = elems[g];
            const float4 p1 = pos[v.x], p2 = pos[v.y], p3 = pos[v.z];
            const float4 p4 = d.kind == KIND_TRI ? f4(0, 0, 0, 0) : pos[v.w];
            const float4 n = is.rot_identity ? enrm_id[g] : enrm[g];
            float kind_bits, rot_bits;
            const int kind = d.kind, rot = is.rot_identity ? 1 : 0;
            std::memcpy(&kind_bits, &kind, 4);
            std::memcpy(&rot_bits, &rot, 4);
            lelems.push_back(f4(p1.x, p1.y, p1.z, p2.x));
            lelems.push_back(f4(p2.y, p2.z, p3.x, p3.y));
            lelems.push_back(f4(p3.z, n.x, n.y, n.z));
            lelems.push_back(f4(area, rot_bits, kind_bits, 0));
            lelems.push_back(f4(p4.x, p4.y, p4.z, 0));
        }
    }
    if (lelems.empty()) lelems.assign(5, f4(0, 0, 0, 0));
    std::vector<float> srgb, bytes;
    build_luts(srgb, bytes);

    DScene& S = c->S;
    // one zero record past the last primitive: prim_step reads the record after a leaf's last
    for (int q = 0; q < 4; q++) prims.push_back(f4(0, 0, 0, 0));
    std::vector<DNode> nodes;
    if (!c->wide) {
        nodes = tlas;
        nodes.insert(nodes.end(), blas.begin(), blas.end());
    }
    // traversal stack entries carry a 24-bit node / instance index (IDX_MASK)
    if (nodes.size() > IDX_MASK || (size_t)scene->ninstances > IDX_MASK)
        return bail(jt::fail(JT_ERR_UNSUPPORTED, "scene exceeds 2^24 BVH nodes or instances"));
    if ((st = upload(c, nodes, &S.nodes)) || (st = upload(c, wnodes, &S.wnodes)) || (st = upload(c, prims, &S.prims)) ||
        (st = upload(c, itrav, &S.inst_trav)) || (st = upload(c, iblas, &S.inst_blas)) || (st = upload(c, ishade, &S.inst_shade)) ||
        (st = upload(c, shapes, &S.shapes)) || (st = upload(c, pos, &S.pos)) || (st = upload(c, nrm, &S.nrm)) ||
        (st = upload(c, tc, &S.tc)) || (st = upload(c, col, &S.col)) || (st = upload(c, elems, &S.elems)) ||
        (st = upload(c, enrm, &S.enrm)) || (st = upload(c, enrm_id, &S.enrm_id)) ||
        (st = upload(c, mats, &S.materials)) || (st = upload(c, texs, &S.textures)) || (st = upload(c, texb, &S.texb)) ||
        (st = upload(c, texf, &S.texf)) || (st = upload(c, envs, &S.envs)) || (st = upload(c, dl, &S.lights)) || (st = upload(c, lhit, &S.light_hit)) || (st = upload(c, lelems, &S.light_elems)) ||
        (st = upload(c, cdf, &S.cdf)) || (st = upload(c, guide_t, &S.guide_t)) || (st = upload(c, guide_a, &S.guide_a)) || (st = upload(c, alias, &S.alias)) || (st = upload(c, srgb, &S.srgb_lut)) || (st = upload(c, bytes, &S.byte_lut)))
        return bail(st);
    S.tlas_nnodes = (int)tlas.size();
    S.tlas_wnodes = tlas_wnodes;
    S.order_flip = params->traversal == JT_TRAVERSAL_REFERENCE ? 0 : 7;  // near and wide: near child first
    S.nenvs = scene->nenvironments;
    S.nlights = lights->nlights;
    S.light_pick_pdf = lights->nlights > 0 ? (float)(1.0 / (double)lights->nlights) : 0.0f;
    // Inline light queries: when every instance light's shape BVH is one leaf (cornellbox's and
    // bathroom1's two-triangle lights, features2's quads), each intersect_instance_bvh of
    // sample_lights_pdf is an instance visit, one box test and at most four primitive tests, so the
    // lane runs its whole light chain where the chain starts (jtk::light_chain) instead of through
    // the traversal loop. Option light_inline=0 turns it off (A/B runs); results are identical.
    {
        bool inl = true;
        for (int k = 0; k < lights->nlights; k++) {
            const int i0 = lights->lights[k].instance;
            if (i0 < 0) continue;
            const jt_bvh_tree& t = bvh->blas[scene->instances[i0].shape];
            inl = inl && t.nnodes > 0 && !t.nodes[0].internal;
        }
        const char* li = opt("light_inline");
        if (li && std::atoi(li) == 0) inl = false;
        S.light_inline = inl ? 1 : 0;
    }

    // ------------------------------------------------------------- small-scene LDS blob
    {
        std::vector<uint4> blob;
        auto add = [&](const void* data, size_t bytes) {
            const int off = (int)blob.size();
            const size_t n16 = (bytes + 15) / 16;
            blob.resize(blob.size() + std::max<size_t>(1, n16));
            if (bytes) std::memcpy(blob.data() + off, data, bytes);
            return off;
        };
        S.o_nodes = add(nodes.data(), nodes.size() * sizeof(DNode));
        S.o_wnodes = add(wnodes.data(), wnodes.size() * sizeof(DWide));
        S.o_prims = add(prims.data(), prims.size() * sizeof(float4));
        S.o_inst_trav = add(itrav.data(), itrav.size() * sizeof(DInstTrav));
        S.o_inst_blas = add(iblas.data(), iblas.size() * sizeof(int4));
        S.o_inst_shade = add(ishade.data(), ishade.size() * sizeof(DInstShade));
        S.o_shapes = add(shapes.data(), shapes.size() * sizeof(DShape));
        S.o_pos = add(pos.data(), pos.size() * sizeof(float4));
        S.o_nrm = add(nrm.data(), nrm.size() * sizeof(float4));
        S.o_tc = add(tc.data(), tc.size() * sizeof(float2));
        S.o_col = add(col.data(), col.size() * sizeof(float4));
        S.o_elems = add(elems.data(), elems.size() * sizeof(int4));
        S.o_enrm = add(enrm.data(), enrm.size() * sizeof(float4));
        S.o_enrm_id = add(enrm_id.data(), enrm_id.size() * sizeof(float4));
        S.o_materials = add(mats.data(), mats.size() * sizeof(DMaterial));
        S.o_lights = add(dl.data(), dl.size() * sizeof(DLight));
        S.o_cdf = add(cdf.data(), cdf.size() * sizeof(float));
        S.o_light_hit = add(lhit.data(), lhit.size() * sizeof(int4));
        S.o_light_elems = add(lelems.data(), lelems.size() * sizeof(float4));
        // LDS mode only when the blob does not cost workgroups per CU: the kernel holds at most
        // 4 workgroups per CU (4 waves/SIMD), so the blob + stack + accumulators may use up to
        // 160 KiB / 4, or as much as HBM mode's stack + accumulators already cost. Override
        // with the option lds_scene=0 (off) or a byte budget for the blob.
        size_t budget = 48 * 1024;
        if (const char* v = opt("lds_scene")) budget = (size_t)std::atoll(v);
        // HBM mode's stack is the kernel's static ring (16 or 32 entries); LDS mode's, without
        // overflow, just the scene's bound
        // + the texel-decode LUTs a texture kernel keeps in LDS (trace_body)
        const size_t acc_bytes = (size_t)ACC_SLOTS * BLOCK * 4 + ((c->feat & FT_TEX) ? 2048 : 0);
        const size_t base_bytes = (size_t)(c->stack <= 16 ? 16 : c->ring) * BLOCK * 4 + acc_bytes;
        const size_t lds_base = lds_stack_bytes(c->stack > 16, c->ring, c->stack) + acc_bytes;
        const size_t bytes = blob.size() * 16;
        const size_t lds_cu = 160 * 1024;
        const size_t wg_hbm = std::min<size_t>(4, lds_cu / base_bytes), wg_lds = lds_cu / (lds_base + bytes);
        S.blob = nullptr;
        S.blob_n16 = 0;
        if (bytes <= budget && wg_lds >= wg_hbm) {
            std::vector<uint4> b(blob);
            if ((st = upload(c, b, &S.blob))) return bail(st);
            S.blob_n16 = (int)blob.size();
        }
        c->lds_scene_bytes = S.blob_n16 ? bytes : 0;
    }
    // auto: wide for a scene in HBM mode whose BVH is deep (a stack bound above 32: bathroom1 46,
    // ecosys 43: +20 %, +30 % over near); near otherwise — features2 (bound 24) runs 2737/2742
    // Mrays/s near vs 2677/2646 wide at 512 spp (gpurun_out/r04m), cornellbox runs from LDS
    if (params->traversal == JT_TRAVERSAL_AUTO && !S.blob_n16 && need > JT_AUTO_WIDE_MIN_STACK) {
        // HBM mode: the wide records (the binary nodes stay uploaded, unused); the instances'
        // BLAS roots become root records
        if ((st = build_all_wide()) != JT_OK) return bail(st);
        for (int k0 = 0; k0 < scene->ninstances; k0++) iblas[inst_new[k0]].x = wroot[scene->instances[k0].shape];
        if ((st = upload(c, wnodes, &S.wnodes)) || (st = upload(c, iblas, &S.inst_blas))) return bail(st);
        S.tlas_wnodes = tlas_wnodes;
        c->wide = true;
    }
    c->traversal = params->traversal == JT_TRAVERSAL_AUTO ? (c->wide ? JT_TRAVERSAL_WIDE : JT_TRAVERSAL_NEAR)
                                                          : params->traversal;
    S.ovf = nullptr;
    S.ovf_stride = 0;
    S.ring = c->ring;
    S.stack_need = c->stack;
    // option test_lds_ring (tests only): use fewer ring entries than allocated, to exercise the overflow
    if (const char* r = opt("test_lds_ring")) {
        int v = std::atoi(r);
        if (v >= 1 && v <= 16 && (v & (v - 1)) == 0) {
            S.ring = v;
            c->stack = std::max(c->stack, 17);  // force the overflow-capable kernel
            c->ring = 16;
        }
    }
    if (c->stack > 16) {  // HBM overflow of the LDS stack ring: `need` entries per lane of the
        // persistent grid (at most 8 workgroups of BLOCK lanes per CU resident; kernel slot
        // blockIdx.x * BLOCK + threadIdx.x: a query never outlives its lane)
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, params->device) != hipSuccess || ncu < 1)
            ncu = 256;
        void* p = nullptr;
        const size_t bytes = (size_t)ncu * 8 * BLOCK * (size_t)need * 4;
        if ((e = hipMalloc(&p, bytes)) != hipSuccess) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc stack overflow"));
        c->allocations.push_back(p);
        S.ovf = (int*)p;
        S.ovf_stride = need;
    }

    DParams& P = c->P;
    const jt_camera& cam = scene->cameras[params->camera];
    std::memcpy(P.cam.frame, cam.frame, sizeof(P.cam.frame));
    P.cam.orthographic = cam.orthographic;
    P.cam.lens = cam.lens;
    P.cam.film = cam.film;
    P.cam.aspect = (params->width > 0 && params->height > 0) ? (float)W / (float)H : cam.aspect;
    // film = aspect >= 1 ? (film, film / aspect) : (film * aspect, film) (src/scene.jl:377-378)
    P.cam.film_x = P.cam.aspect >= 1 ? cam.film : cam.film * P.cam.aspect;
    P.cam.film_y = P.cam.aspect >= 1 ? cam.film / P.cam.aspect : cam.film;
    P.cam.focus = cam.focus;
    P.cam.aperture = cam.aperture;
    P.cam.pinhole = (std::signbit(cam.aperture) == 0 && cam.aperture == 0.0f) ? 1 : 0;
    P.width = W;
    P.height = H;
    P.bounces = params->bounces;
    P.sampler = params->sampler;
    P.clamp = (float)params->clamp;
    P.envhidden = params->envhidden;
    P.tentfilter = params->tentfilter;
    P.nocaustics = params->nocaustics;
    P.first = 0;
    P.seed = params->seed;
    P.tile_stride = 1;  // every tile (jt_create_multi may split by tiles)
    P.tile_offset = 0;
    // option tile_share "stride,offset": trace only tiles offset, offset + stride, ... — one
    // process's share of a render split by tiles over one process per GPU (bench.py), or one
    // device's share of jt_create_multi's tile split reproduced on one GPU (tests)
    if (const char* ts = opt("tile_share")) {
        int k = 0, o = 0;
        if (std::sscanf(ts, "%d,%d", &k, &o) == 2 && k >= 1 && o >= 0 && o < k) {
            P.tile_stride = k;
            P.tile_offset = o;
        }
    }
    // sample streams: from the pixels this context traces (a tile share traces 1/stride of them)
    c->lk = stream_log2(((long long)W * H + P.tile_stride - 1) / P.tile_stride, std::max(1, params->batch));
    bool forced_streams = false;
    if (const char* ks = opt("streams")) {
        forced_streams = true;
        const int k = std::atoi(ks);
        if (k < 1 || k > JT_MAX_STREAMS || (k & (k - 1)) != 0)
            return bail(jt::fail(JT_ERR_INVALID, "option streams: a power of two in [1, " + std::to_string(JT_MAX_STREAMS) + "]"));
        c->lk = 0;
        while ((1 << c->lk) < k) c->lk++;
    }
    P.lk = c->lk;
    // measured best (cornellbox): 40 waiting lanes per shading phase; 48 with
    // light-hit steps in the traversal phase (they take the light queries out of the phases)
    bool inst_light = false;  // sample_lights_pdf runs instance queries (light-hit steps can run)
    for (int k = 0; k < lights->nlights; k++) inst_light |= lights->lights[k].instance >= 0;
    c->kmask = kernel_mask(c->feat, c->stack, c->ring, c->lds_scene_bytes > 0, c->S.light_inline != 0, inst_light);
    // light queries leave the shading phase's waiting lanes early (light-hit steps) or never wait
    // there at all (inline chains): the gate then waits for more lanes
    const int smp = c->sampler == JT_SAMPLER_NAIVE ? 2 : 1;
    const bool lstep = inst_light && smp == 1 && (light_steps(smp, c->kmask) || c->S.light_inline);
    // deep BVHs (stack bound > 32: bathroom1, ecosys) shade sooner: their lanes finish queries far
    // apart, so waiting for many leaves the wave idle. Re-swept in round 4 (per-lane work items,
    // short chunks, auto traversal; profiles/r04_ab/wait_lanes_r04o.txt): cornellbox 56 (52
    // even, 48 / 60 -1.3 %, 64 -6 %), features2 56 (60 -2.9 %, 48 -0.5 %, 64 -9 %), bathroom1 40
    // (48 even, 24 -10 %), ecosys (no instance lights) 24 (16 -1.2 %, 32 -2.2 %, 8 -11 %)
    const bool deep = c->stack > 32;
    P.wait_lanes = lstep ? (deep ? 40 : 56) : deep ? 24 : 40;
    if (const char* wl = opt("wait_lanes")) P.wait_lanes = std::max(1, std::min(64, std::atoi(wl)));
    P.light_lanes = 2;
    if (const char* ll = opt("light_lanes")) P.light_lanes = std::max(1, std::min(65, std::atoi(ll)));

    // accumulators (make_trace_state: zeroed) + counters
    const size_t np = (size_t)W * (size_t)H;
    void *img, *alb, *nrmb, *hits, *cnt;
    if ((e = hipMalloc(&img, np * 16)) != hipSuccess) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc accumulators"));
    c->allocations.push_back(img);
    if ((e = hipMalloc(&alb, np * 16)) != hipSuccess) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc accumulators"));
    c->allocations.push_back(alb);
    if ((e = hipMalloc(&nrmb, np * 16)) != hipSuccess) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc accumulators"));
    c->allocations.push_back(nrmb);
    if ((e = hipMalloc(&hits, np * 8)) != hipSuccess) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc accumulators"));
    c->allocations.push_back(hits);
    if ((e = hipMalloc(&cnt, 32 * 8)) != hipSuccess) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc counters"));
    c->allocations.push_back(cnt);
    // persistent scheduling: unit counters (zeroed before each launch)
    c->tiles = ((W + 7) / 8) * ((H + 7) / 8);
    if (c->tiles >= (1 << 20))  // the per-lane work items address a pixel as tile * 64 + l
        return bail(jt::fail(JT_ERR_UNSUPPORTED, "image above 2^20 8x8 tiles (67 Mpixels)"));
    void* sched = nullptr;
    if ((e = hipMalloc(&sched, SCHED_BYTES)) != hipSuccess) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc schedule"));
    c->allocations.push_back(sched);
    // the sample streams' means (k > 1): image, albedo + hits, normal per (stream, slot of the
    // launch's tiles: a tile share holds only its own pixels). Too little memory for k streams
    // halves k (the image bits then follow the smaller k, jt_get_streams) unless the option
    // "streams" asked for this k.
    void* part[3] = {nullptr, nullptr, nullptr};
    const size_t nslot = (size_t)launch_tiles(P) * 64;
    while (c->lk > 0) {
        bool ok = true;
        for (int k = 0; k < 3 && ok; k++) ok = hipMalloc(&part[k], nslot * 16 << c->lk) == hipSuccess;
        if (ok) break;
        (void)hipGetLastError();
        for (int k = 0; k < 3; k++) {
            if (part[k]) (void)hipFree(part[k]);
            part[k] = nullptr;
        }
        if (forced_streams) return bail(jt::fail(JT_ERR_NOMEM, "hipMalloc stream means"));
        c->lk--;
    }
    for (int k = 0; k < 3; k++)
        if (part[k]) c->allocations.push_back(part[k]);
    P.lk = c->lk;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, params->device) == hipSuccess && cus > 0) c->cus = cus;
    c->A = DAccum{(float4*)img, (float4*)alb, (float4*)nrmb, (long long*)hits, (unsigned long long*)cnt, (unsigned*)sched,
                  (float4*)part[0], (float4*)part[1], (float4*)part[2], (int)nslot};
    st = jt_reset(c);
    if (st != JT_OK) return bail(st);
    *out = c;
    return JT_OK;
}

int jt_create_multi(const jt_scene* scene, const jt_scene_bvh* bvh, const jt_lights* lights, const jt_params* params,
                    const int32_t* devices, int32_t ndevices, jt_ctx** out) {
    if (!out) return jt::fail(JT_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (!params) return jt::fail(JT_ERR_INVALID, "NULL argument");
    int avail = 0;
    if (hipGetDeviceCount(&avail) != hipSuccess) avail = 0;
    if (ndevices < 1 || ndevices > avail)
        return jt::fail(JT_ERR_INVALID, "ndevices must be in [1, " + std::to_string(avail) + "]");
    std::vector<int> devs(ndevices);
    for (int d = 0; d < ndevices; d++) {
        devs[d] = devices ? devices[d] : d;
        if (devs[d] < 0 || devs[d] >= avail) return jt::fail(JT_ERR_INVALID, "device id out of range");
        for (int k = 0; k < d; k++)
            if (devs[k] == devs[d]) return jt::fail(JT_ERR_INVALID, "a device is listed twice");
    }
    if (!rccl().ok) return jt::fail(JT_ERR_UNSUPPORTED, "librccl.so.1 (RCCL) could not be loaded");
    jt_ctx* c = new jt_ctx();
    for (int d = 0; d < ndevices; d++) {
        jt_params p = *params;
        p.device = devs[d];
        jt_ctx* s = nullptr;
        const int st = jt_create(scene, bvh, lights, &p, &s);
        if (st != JT_OK) {
            jt_destroy(c);
            return st;
        }
        c->sub.push_back(s);
    }
    c->nsub.assign(ndevices, 0);
    // split mode (jt_ctx::tile_split); the option multi_split=tiles|samples overrides
    c->tile_split = params->batch < ndevices;
    {
        const auto opts = jt::options_snapshot();
        const auto m = opts.find("multi_split");
        if (m != opts.end() && m->second == "tiles") c->tile_split = true;
        if (m != opts.end() && m->second == "samples") c->tile_split = false;
    }
    // every sub-context traces every tile under the sample split (a tile_share option never
    // leaves tiles out of the reduced image), its interleaved share under the tile split
    for (int d = 0; d < ndevices; d++) {
        c->sub[d]->P.tile_stride = c->tile_split ? ndevices : 1;
        c->sub[d]->P.tile_offset = c->tile_split ? d : 0;
        // a device's share leaves the other devices' tiles at zero for the summing reduce
        const int st = c->tile_split ? zero_if_stale(c->sub[d]) : JT_OK;
        if (st != JT_OK) {
            jt_destroy(c);
            return st;
        }
    }
    c->comms.resize(ndevices);
    ncclResult_t r = rccl().CommInitAll(c->comms.data(), ndevices, devs.data());
    if (r != ncclSuccess) {
        c->comms.clear();
        jt_destroy(c);
        return nccl_fail(r, "ncclCommInitAll");
    }
    jt_ctx* s0 = c->sub[0];
    c->device = s0->device;
    c->width = s0->width;
    c->height = s0->height;
    c->total_samples = s0->total_samples;
    c->batch = s0->batch;
    c->sampler = s0->sampler;
    (void)hipSetDevice(s0->device);
    const size_t np = (size_t)c->width * c->height;
    if (hipMalloc(&c->red, np * 16) != hipSuccess || hipMalloc(&c->red_hits, np * 8) != hipSuccess) {
        jt_destroy(c);
        return jt::fail(JT_ERR_NOMEM, "hipMalloc reduce buffers");
    }
    *out = c;
    return JT_OK;
}

namespace {
int zero_if_stale(jt_ctx* c) {
    if (!c->stale) return JT_OK;
    (void)hipSetDevice(c->device);
    const size_t np = (size_t)c->width * (size_t)c->height;
    hipError_t e;
    if ((e = hipMemsetAsync(c->A.image, 0, np * 16, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->A.albedo, 0, np * 16, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->A.normal, 0, np * 16, c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->A.hits, 0, np * 8, c->stream)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync");
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    c->stale = false;
    return JT_OK;
}
// the deferred AOV combine of the last launch (jt_ctx::aov_pending), before albedo, normal or
// hits are read: jt_get_aovs, jt_synchronize, jt_get_device_buffers
int finish_aovs(jt_ctx* c) {
    if (!c->aov_pending) return JT_OK;
    (void)hipSetDevice(c->device);
    const int nblk = (int)(((long long)launch_tiles(c->P) * 64 + 255) / 256);
    hipLaunchKernelGGL(jtk::combine_kernel<true>, dim3(nblk), dim3(256), 0, c->stream, c->P, c->A, c->aov_cw);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        c->failed = true;
        return hip_fail(e, "AOV combine");
    }
    c->aov_pending = false;
    return JT_OK;
}
}  // namespace

int jt_reset(jt_ctx* c) {
    if (!c) return jt::fail(JT_ERR_INVALID, "ctx is NULL");
    if (!c->sub.empty()) {
        for (jt_ctx* s : c->sub) {
            const int st = jt_reset(s);
            if (st != JT_OK) return st;
        }
        std::fill(c->nsub.begin(), c->nsub.end(), 0LL);
        c->pend0 = c->pend1 = 0;  // deferred samples are dropped with the state
        c->first = -1;
        c->next = 0;
        c->failed = false;
        c->launches = 0;
        c->kernel_ms = 0;
        return JT_OK;
    }
    (void)hipSetDevice(c->device);
    hipError_t e;
    // a failed flush may have left chains queued on stream2 (a complete one ends on `stream`)
    if (c->stream2 && (e = hipStreamSynchronize(c->stream2)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    if ((e = hipMemsetAsync(c->A.counters, 0, 256, c->stream)) != hipSuccess) return hip_fail(e, "hipMemsetAsync");
    // make_trace_state's zeroed buffers (src/trace.jl:189-213). A context that traces every tile
    // overwrites every pixel in its first launch without reading it (a stream's first sample
    // starts from zero), so they are zeroed only if read before that launch (zero_if_stale); a
    // tile share keeps the other tiles' pixels at zero for the reduce, and a context whose device
    // buffers were handed out is read in place, so those zero them now.
    c->stale = true;
    c->aov_pending = false;
    c->pend0 = c->pend1 = 0;  // deferred samples are dropped with the state
    // a caller holding the device pointers (jt_get_device_buffers) sees the zeros at once
    if (c->P.tile_stride != 1 || c->exported) {
        const int st = zero_if_stale(c);
        if (st != JT_OK) return st;
    }
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    c->first = -1;
    c->next = 0;
    c->failed = false;
    c->launches = 0;
    c->kernel_ms = 0;
    return JT_OK;
}

}  // extern "C"

namespace {
// the chunk size of a one-stream context: as many one-sample streams as two sets of stream-mean
// buffers hold, at most 64 (JT_MAX_STREAMS) and 2^27 (stream, slot) records in all (6.4 GB);
// allocated at the first multi-sample range, halved on NOMEM. 0 after jt_create (none yet), 1:
// none possible (the range then runs as one launch of long items).
int ensure_chunk(jt_ctx* c) {
    if (c->chunk) return JT_OK;
    const long long nslot = (long long)launch_tiles(c->P) * 64;
    int m = JT_MAX_STREAMS;
    while (m > 1 && 2 * nslot * m > JT_STREAM_ITEMS_MAX) m >>= 1;
    (void)hipSetDevice(c->device);
    if (hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess) {
        c->stream2 = nullptr;
        m = 1;
    }
    for (int k = 0; k < 2 && m > 1; k++)
        if (hipEventCreateWithFlags(&c->trace_done[k], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->chain_done[k], hipEventDisableTiming) != hipSuccess)
            m = 1;
    for (; m > 1; m >>= 1) {
        void* part[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        bool ok = true;
        for (int k = 0; k < 6 && ok; k++) ok = hipMalloc(&part[k], (size_t)nslot * 16 * (size_t)m) == hipSuccess;
        if (ok) {
            for (int k = 0; k < 6; k++) {
                c->allocations.push_back(part[k]);
                c->cpart[k / 3][k % 3] = (float4*)part[k];
            }
            break;
        }
        (void)hipGetLastError();
        for (int k = 0; k < 6; k++)
            if (part[k]) (void)hipFree(part[k]);
    }
    c->chunk = m;
    return JT_OK;
}

// enqueue the trace launch of global samples [s0, s1) for local samples starting at `first`
// (stream t & (k-1) of local sample t = s - first, DParams::lk), then — with k > 1 — the combine
// of every pixel's stream means into the image and AOV buffers
int launch_range(jt_ctx* c, const DParams& P, const DAccum& A, int32_t s0, int32_t s1) {
    hipError_t e = hipMemsetAsync(c->A.work, 0, SCHED_BYTES, c->stream);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync schedule");
    if (c->sampler == JT_SAMPLER_NAIVE)
        e = c->count ? launch_s<2, 1>(c->stack, c->ring, c->kmask, c->wide, c->S, P, s0, s1, A, c->stream, c->cus)
                     : launch_s<2, 0>(c->stack, c->ring, c->kmask, c->wide, c->S, P, s0, s1, A, c->stream, c->cus);
    else
        e = c->count ? launch_s<1, 1>(c->stack, c->ring, c->kmask, c->wide, c->S, P, s0, s1, A, c->stream, c->cus)
                     : launch_s<1, 0>(c->stack, c->ring, c->kmask, c->wide, c->S, P, s0, s1, A, c->stream, c->cus);
    if (e != hipSuccess) return hip_fail(e, "trace kernel launch");
    return JT_OK;
}

// enqueue the launches of global samples [s0, s1) of a context whose local samples start at
// `first`. k > 1 streams: one trace launch + the combine. k = 1 (the reference's single running
// mean): one launch for one sample; a longer range in chunks (jt_ctx::chunk) of one-sample streams,
// each folded into the running mean by chain_kernel — the bits of one launch per sample, with
// m times the items per launch
int trace_launch(jt_ctx* c, int32_t s0, int32_t s1, int32_t first) {
    (void)hipSetDevice(c->device);
    hipError_t e;
    if ((e = hipEventRecord(c->ev0, c->stream)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    const int tiles = launch_tiles(c->P);
    const int nblk = (int)(((long long)tiles * 64 + 255) / 256);
    int launches = 0;
    if (c->lk == 0 && s1 - s0 > 1 && ensure_chunk(c) == JT_OK && c->chunk > 1) {
        // chunk i traces into buffer set i & 1 on `stream`; its chain runs on `stream2` after that
        // trace and after chain i - 1 (stream order), overlapping trace i + 1; trace i + 2 reuses
        // the set once chain i has read it. `stream` then waits for the last chain (ev1 covers it).
        int i = 0;
        for (int32_t x = s0; x < s1; x += c->chunk, i++) {
            const int32_t y = std::min(s1, x + c->chunk);
            const int set = i & 1;
            DParams P = c->P;  // the chunk's samples as one-sample streams x .. y-1
            P.first = x;
            P.lk = 0;
            while ((1 << P.lk) < y - x) P.lk++;
            DAccum A = c->A;
            A.part_img = c->cpart[set][0];
            A.part_alb = c->cpart[set][1];
            A.part_nrm = c->cpart[set][2];
            A.nslot = tiles * 64;
            if (i >= 2 && (e = hipStreamWaitEvent(c->stream, c->chain_done[set], 0)) != hipSuccess)
                return hip_fail(e, "hipStreamWaitEvent");
            if (const int st = launch_range(c, P, A, x, y)) return st;
            if ((e = hipEventRecord(c->trace_done[set], c->stream)) != hipSuccess ||
                (e = hipStreamWaitEvent(c->stream2, c->trace_done[set], 0)) != hipSuccess)
                return hip_fail(e, "hipEventRecord");
            if (nblk > 0) hipLaunchKernelGGL(chain_kernel, dim3(nblk), dim3(256), 0, c->stream2, c->P, A, x - first, y - x);
            if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "chain kernel launch");
            if ((e = hipEventRecord(c->chain_done[set], c->stream2)) != hipSuccess) return hip_fail(e, "hipEventRecord");
            launches++;
        }
        if ((e = hipStreamWaitEvent(c->stream, c->chain_done[(i - 1) & 1], 0)) != hipSuccess)
            return hip_fail(e, "hipStreamWaitEvent");
    } else {
        c->P.first = first;
        if (const int st = launch_range(c, c->P, c->A, s0, s1)) return st;
        launches = 1;
        if (c->lk > 0) {
            // weights n_j / n of the streams after this launch: n local samples, stream j holds
            // those t < n with t mod k == j (include/jtrace.h jt_get_streams restates the rule)
            const long long n = (long long)s1 - first, k = 1LL << c->lk;
            DCombine cw{};
            cw.ns = (int)std::min(n, k);
            for (int j = 0; j < cw.ns; j++) cw.w[j] = (float)((double)((n - 1 - j) / k + 1) / (double)n);
            if (nblk > 0) hipLaunchKernelGGL(combine_kernel<false>, dim3(nblk), dim3(256), 0, c->stream, c->P, c->A, cw);
            if ((e = hipGetLastError()) != hipSuccess) return hip_fail(e, "combine kernel launch");
            c->aov_pending = nblk > 0;
            c->aov_cw = cw;
        }
    }
    if ((e = hipEventRecord(c->ev1, c->stream)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    c->launches += launches - 1;  // trace_finish counts one
    c->stale = false;  // every pixel of the launch's tiles was written (tile shares were zeroed at reset)
    return JT_OK;
}
// wait for the launch; its device time in *ms
int trace_finish(jt_ctx* c, float* ms) {
    (void)hipSetDevice(c->device);
    hipError_t e;
    if ((e = hipEventSynchronize(c->ev1)) != hipSuccess) return hip_fail(e, "trace kernel");
    *ms = 0;
    (void)hipEventElapsedTime(ms, c->ev0, c->ev1);
    c->kernel_ms += *ms;
    c->launches++;
    return JT_OK;
}

// multi-device trace_samples step. Sample split: [s0, s1) in contiguous shares, one per device,
// each appended to that device's own running mean (weight 1/(n_d + k + 1) for its k-th new
// sample). Tile split: every device traces all of [s0, s1) on its own tiles (the running-mean
// weights are the single-device ones: first = the context's first sample).
int multi_trace_range(jt_ctx* c, int32_t s0, int32_t s1) {
    const int D = (int)c->sub.size();
    const long long L = s1 - s0;
    std::vector<int> a(D), b(D);
    std::vector<char> launched(D, 0);
    int status = JT_OK;
    for (int d = 0; d < D && status == JT_OK; d++) {
        a[d] = c->tile_split ? s0 : s0 + (int)(L * d / D);
        b[d] = c->tile_split ? s1 : s0 + (int)(L * (d + 1) / D);
        if (a[d] < b[d]) {
            const int32_t first = c->tile_split ? c->first : (int32_t)(a[d] - c->nsub[d]);
            status = trace_launch(c->sub[d], a[d], b[d], first);
            launched[d] = status == JT_OK;
        }
    }
    // wait for every launch already queued, even after a failed one: they add to their devices'
    // running means, so the context is unusable (failed) unless all of them ran
    float wall = 0;
    for (int d = 0; d < D; d++) {
        if (!launched[d]) continue;
        float ms = 0;
        const int st = trace_finish(c->sub[d], &ms);
        if (st != JT_OK && status == JT_OK) status = st;
        c->nsub[d] += b[d] - a[d];
        wall = std::max(wall, ms);
    }
    if (status != JT_OK) {
        c->failed = true;
        return status;
    }
    c->kernel_ms += wall;  // the launches run concurrently: the slowest device's time
    c->launches++;
    c->next = s1;
    return JT_OK;
}

// the reduce of the devices' running means onto device 0, then to the host. Sample split: one
// RCCL reduce with a per-rank premultiplied sum, sum_d mean_d * n_d / N; tile split: the devices'
// pixels are disjoint (zero elsewhere), so a plain sum. which: 0 image, 1 albedo, 2 normal
// (float4 buffers); hits (int64) are summed.
int multi_reduce(jt_ctx* c, int which, float* out4, int64_t* hits) {
    const int D = (int)c->sub.size();
    const size_t np = (size_t)c->width * c->height;
    long long N = 0;
    for (long long n : c->nsub) N += n;
    // the premultiplied-sum ops created so far, destroyed on every exit path
    struct Ops {
        jt_ctx* c;
        std::vector<ncclRedOp_t> op;
        ~Ops() {
            for (size_t d = 0; d < op.size(); d++) (void)rccl().RedOpDestroy(op[d], c->comms[d]);
        }
    } ops{c, {}};
    std::vector<float> w(D);
    ncclResult_t r;
    if (out4 && !c->tile_split) {
        for (int d = 0; d < D; d++) {
            w[d] = N > 0 ? (float)((double)c->nsub[d] / (double)N) : (d == 0 ? 1.0f : 0.0f);
            ncclRedOp_t op;
            if ((r = rccl().RedOpCreatePreMulSum(&op, &w[d], ncclFloat32, ncclScalarHostImmediate, c->comms[d])) != ncclSuccess)
                return nccl_fail(r, "ncclRedOpCreatePreMulSum");
            ops.op.push_back(op);
        }
    }
    if ((r = rccl().GroupStart()) != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
    for (int d = 0; d < D; d++) {
        jt_ctx* s = c->sub[d];
        (void)hipSetDevice(s->device);
        if (out4) {
            const float4* src = which == 0 ? s->A.image : which == 1 ? s->A.albedo : s->A.normal;
            r = rccl().Reduce(src, d == 0 ? (void*)c->red : (void*)src, np * 4, ncclFloat32,
                              c->tile_split ? ncclSum : ops.op[d], 0, c->comms[d], s->stream);
        } else {
            r = rccl().Reduce(s->A.hits, d == 0 ? (void*)c->red_hits : (void*)s->A.hits, np, ncclInt64, ncclSum, 0, c->comms[d],
                              s->stream);
        }
        if (r != ncclSuccess) {
            (void)rccl().GroupEnd();
            return nccl_fail(r, "ncclReduce");
        }
    }
    if ((r = rccl().GroupEnd()) != ncclSuccess) return nccl_fail(r, "ncclGroupEnd");
    hipError_t e;
    for (int d = 0; d < D; d++) {
        (void)hipSetDevice(c->sub[d]->device);
        if ((e = hipStreamSynchronize(c->sub[d]->stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    }
    (void)hipSetDevice(c->sub[0]->device);
    if (out4) e = hipMemcpy(out4, c->red, np * 16, hipMemcpyDeviceToHost);
    else e = hipMemcpy(hits, c->red_hits, np * 8, hipMemcpyDeviceToHost);
    return e == hipSuccess ? JT_OK : hip_fail(e, "hipMemcpy reduce");
}

// trace the deferred samples [pend0, pend1) (jt_ctx) and wait for them; every call that reads
// the context's results or device buffers runs this first
int flush(jt_ctx* c) {
    if (c->pend1 <= c->pend0) return JT_OK;
    const int32_t s0 = c->pend0, s1 = c->pend1;
    c->pend0 = c->pend1 = 0;
    if (!c->sub.empty()) return multi_trace_range(c, s0, s1);
    int st = trace_launch(c, s0, s1, c->first);
    float ms = 0;
    if (st == JT_OK) st = trace_finish(c, &ms);
    if (st != JT_OK) c->failed = true;
    return st;
}
}  // namespace

extern "C" {

int jt_trace_range(jt_ctx* c, int32_t s0, int32_t s1) {
    if (!c) return jt::fail(JT_ERR_INVALID, "ctx is NULL");
    if (s0 < 0 || s1 < s0) return jt::fail(JT_ERR_STATE, "invalid sample range");
    if (s0 == s1) return JT_OK;
    if (c->failed) return jt::fail(JT_ERR_STATE, "a previous launch failed; jt_reset the context");
    if (c->first >= 0 && s0 != c->next)
        return jt::fail(JT_ERR_STATE, "samples must be accumulated in order (expected " + std::to_string(c->next) + ")");
    if (c->first < 0) c->first = s0;
    // queue the range behind the deferred ones (jt_ctx::pend0); trace them all once enough are
    // queued, the render is complete (params.samples: the end of Jtrace.main's loop), or a caller
    // reads the accumulators in place (jt_get_device_buffers: it sees every range at once)
    if (c->pend1 <= c->pend0) c->pend0 = s0;
    c->pend1 = s1;
    c->next = s1;
    const bool in_place = c->exported || (!c->sub.empty() && c->sub[0]->exported);
    if (in_place || c->pend1 - c->pend0 >= JT_DEFER_SAMPLES || c->next >= c->total_samples) return flush(c);
    return JT_OK;
}

int jt_trace_samples(jt_ctx* c) {
    if (!c) return jt::fail(JT_ERR_INVALID, "ctx is NULL");
    const int n = c->first < 0 ? 0 : c->next;
    if (n >= c->total_samples) return JT_OK;  // state.samples >= params.samples
    const int target = std::min(n + c->batch, c->total_samples);
    return jt_trace_range(c, n, target);
}

int jt_get_streams(const jt_ctx* c, int32_t* streams) {
    if (!c || !streams) return jt::fail(JT_ERR_INVALID, "NULL argument");
    *streams = 1 << (c->sub.empty() ? c->lk : c->sub[0]->lk);
    return JT_OK;
}

int jt_get_samples(const jt_ctx* c, int32_t* samples) {
    if (!c || !samples) return jt::fail(JT_ERR_INVALID, "NULL argument");
    *samples = c->first < 0 ? 0 : c->next - c->first;
    return JT_OK;
}

int jt_get_size(const jt_ctx* c, int32_t* w, int32_t* h) {
    if (!c || !w || !h) return jt::fail(JT_ERR_INVALID, "NULL argument");
    *w = c->width;
    *h = c->height;
    return JT_OK;
}

int jt_get_image(jt_ctx* c, float* rgba) {
    if (!c || !rgba) return jt::fail(JT_ERR_INVALID, "NULL argument");
    if (const int st = flush(c)) return st;
    if (c->failed) return jt::fail(JT_ERR_STATE, "the running means are corrupt (a launch failed); jt_reset the context");
    if (!c->sub.empty()) {
        for (jt_ctx* s : c->sub)
            if (const int st = zero_if_stale(s)) return st;
        return multi_reduce(c, 0, rgba, nullptr);
    }
    if (const int st = zero_if_stale(c)) return st;
    (void)hipSetDevice(c->device);
    hipError_t e = hipMemcpy(rgba, c->A.image, (size_t)c->width * c->height * 16, hipMemcpyDeviceToHost);
    return e == hipSuccess ? JT_OK : hip_fail(e, "hipMemcpy image");
}

int jt_get_aovs(jt_ctx* c, float* albedo, float* normal, int64_t* hits) {
    if (!c) return jt::fail(JT_ERR_INVALID, "ctx is NULL");
    if (const int st = flush(c)) return st;
    if (c->failed) return jt::fail(JT_ERR_STATE, "the running means are corrupt (a launch failed); jt_reset the context");
    for (jt_ctx* s : c->sub)
        if (const int st = zero_if_stale(s)) return st;
    for (jt_ctx* s : c->sub)
        if (const int st = finish_aovs(s)) return st;
    if (c->sub.empty()) {
        if (const int st = zero_if_stale(c)) return st;
        if (const int st = finish_aovs(c)) return st;
    }
    (void)hipSetDevice(c->device);
    const size_t np = (size_t)c->width * c->height;
    std::vector<float4> tmp(np);
    hipError_t e;
    const bool multi = !c->sub.empty();
    int st;
    if (albedo) {
        if (multi) {
            if ((st = multi_reduce(c, 1, reinterpret_cast<float*>(tmp.data()), nullptr)) != JT_OK) return st;
        } else if ((e = hipMemcpy(tmp.data(), c->A.albedo, np * 16, hipMemcpyDeviceToHost)) != hipSuccess) {
            return hip_fail(e, "hipMemcpy");
        }
        for (size_t k = 0; k < np; k++) {
            albedo[3 * k] = tmp[k].x;
            albedo[3 * k + 1] = tmp[k].y;
            albedo[3 * k + 2] = tmp[k].z;
        }
    }
    if (normal) {
        if (multi) {
            if ((st = multi_reduce(c, 2, reinterpret_cast<float*>(tmp.data()), nullptr)) != JT_OK) return st;
        } else if ((e = hipMemcpy(tmp.data(), c->A.normal, np * 16, hipMemcpyDeviceToHost)) != hipSuccess) {
            return hip_fail(e, "hipMemcpy");
        }
        for (size_t k = 0; k < np; k++) {
            normal[3 * k] = tmp[k].x;
            normal[3 * k + 1] = tmp[k].y;
            normal[3 * k + 2] = tmp[k].z;
        }
    }
    if (hits) {
        if (multi) {
            if ((st = multi_reduce(c, 0, nullptr, hits)) != JT_OK) return st;
        } else if ((e = hipMemcpy(hits, c->A.hits, np * 8, hipMemcpyDeviceToHost)) != hipSuccess) {
            return hip_fail(e, "hipMemcpy");
        }
    }
    return JT_OK;
}

int jt_get_counters(jt_ctx* c, jt_counters* out) {
    if (!c || !out) return jt::fail(JT_ERR_INVALID, "NULL argument");
    if (const int st = flush(c)) return st;
    if (!c->sub.empty()) {  // summed over the devices; kernel_ms: per launch the slowest device
        jt_counters sum{};
        for (jt_ctx* s : c->sub) {
            jt_counters k{};
            const int st = jt_get_counters(s, &k);
            if (st != JT_OK) return st;
            sum.paths += k.paths;
            sum.rays += k.rays;
            sum.light_queries += k.light_queries;
            sum.nodes += k.nodes;
            sum.instances += k.instances;
            sum.prims += k.prims;
            sum.shades += k.shades;
        }
        sum.launches = c->launches;
        sum.kernel_ms = c->kernel_ms;
        *out = sum;
        return JT_OK;
    }
    (void)hipSetDevice(c->device);
    unsigned long long v[8] = {0};
    hipError_t e = hipMemcpy(v, c->A.counters, 7 * 8, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy counters");
    out->paths = v[0];
    out->rays = v[1];
    out->light_queries = v[2];
    out->nodes = v[3];
    out->instances = v[4];
    out->prims = v[5];
    out->shades = v[6];
    out->launches = c->launches;
    out->kernel_ms = c->kernel_ms;
    return JT_OK;
}

int jt_get_device_buffers(jt_ctx* c, jt_device_buffers* out) {
    if (!c || !out) return jt::fail(JT_ERR_INVALID, "NULL argument");
    if (const int st = flush(c)) return st;
    if (!c->sub.empty()) return jt_get_device_buffers(c->sub[0], out);  // device 0's share
    if (const int st = zero_if_stale(c)) return st;
    if (const int st = finish_aovs(c)) return st;
    c->exported = true;  // jt_reset now zeroes the buffers at once (the caller may read them)
    out->image = c->A.image;
    out->albedo = c->A.albedo;
    out->normal = c->A.normal;
    out->hits = c->A.hits;
    out->width = c->width;
    out->height = c->height;
    out->stream = c->stream;
    return JT_OK;
}

// diagnostic build only (JT_STAMPS=1): per-phase wave clocks and shading-phase material coherence
// (24 u64), read by scripts/stamps.py
extern "C" int jt_debug_stamps(jt_ctx* c, unsigned long long* out8) {
    if (!c || !out8) return jt::fail(JT_ERR_INVALID, "NULL argument");
    hipError_t e = hipMemcpy(out8, c->A.counters + 8, 24 * 8, hipMemcpyDeviceToHost);
    return e == hipSuccess ? JT_OK : hip_fail(e, "hipMemcpy stamps");
}

int jt_describe(const jt_ctx* c, char* buf, int32_t n) {
    if (!c || !buf || n <= 0) return jt::fail(JT_ERR_INVALID, "NULL argument");
    if (!c->sub.empty()) {
        char tmp[640];
        const int st = jt_describe(c->sub[0], tmp, sizeof tmp);
        if (st != JT_OK) return st;
        std::snprintf(buf, (size_t)n, "%s devices=%d split=%s", tmp, (int)c->sub.size(), c->tile_split ? "tiles" : "samples");
        return JT_OK;
    }
    const bool ovf = c->stack > 16;
    const int ring = ovf ? c->ring : 16;
    // test-only options in effect (jt_set_option): a tile filter, a shortened LDS ring
    char filt[96] = "";
    if (c->P.tile_stride != 1 || c->S.ring != c->ring)
        std::snprintf(filt, sizeof filt, " tile_filter=%d/%d ring_used=%d", c->P.tile_offset, c->P.tile_stride, c->S.ring);
    char tmp[640];
    std::snprintf(tmp, sizeof tmp,
                  "kernel=%s<%d,%d,%s,%d,%d,%s> mode=%s scene_lds_bytes=%zu stack_bound=%d lds_ring=%d hbm_overflow=%d "
                  "wait_lanes=%d light_lanes=%d streams=%d tiles=%d block=%d env_alias=%d light_inline=%d "
                  "traversal=%s%s",
                  c->lds_scene_bytes ? "trace_kernel_lds" : "trace_kernel", c->sampler == JT_SAMPLER_NAIVE ? 2 : 1,
                  ring, ovf ? "true" : "false", c->count, c->kmask, c->wide ? "true" : "false",
                  c->lds_scene_bytes ? "lds" : "hbm", c->lds_scene_bytes,
                  c->stack, ring, ovf ? 1 : 0, c->P.wait_lanes, c->P.light_lanes, 1 << c->lk, c->tiles, BLOCK,
                  c->env_alias ? 1 : 0, c->S.light_inline,
                  c->traversal == JT_TRAVERSAL_REFERENCE ? "reference" : c->traversal == JT_TRAVERSAL_NEAR ? "near" : "wide",
                  filt);
    std::snprintf(buf, (size_t)n, "%s", tmp);
    return JT_OK;
}

int jt_set_counters(jt_ctx* c, int32_t level) {
    if (!c) return jt::fail(JT_ERR_INVALID, "ctx is NULL");
    if (level != 0 && level != 1) return jt::fail(JT_ERR_INVALID, "counter level must be 0 or 1");
    if (const int st = flush(c)) return st;  // queued samples are traced at the level they were queued at
    for (jt_ctx* s : c->sub) s->count = level;
    c->count = level;
    return JT_OK;
}

int jt_synchronize(jt_ctx* c) {
    if (!c) return jt::fail(JT_ERR_INVALID, "ctx is NULL");
    if (const int st = flush(c)) return st;
    for (jt_ctx* s : c->sub) {
        const int st = jt_synchronize(s);
        if (st != JT_OK) return st;
    }
    if (!c->sub.empty()) return JT_OK;
    if (const int st = finish_aovs(c)) return st;
    (void)hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? JT_OK : hip_fail(e, "hipStreamSynchronize");
}

}  // extern "C"
