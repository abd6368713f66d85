// AoS vs SoA for the BVH node records (VERDICT r1 "N2"): a microbenchmark of the
// traversal's access pattern on gfx950. Every lane chases its own dependent chain of node
// fetches (the next index comes from the node just read, as a stack pop's does), over a node
// array sized like a large scene's BVH (L2/MALL-resident) or like cornellbox's (L1-resident).
// Each fetch reads the 32 B of one node (6 bounds + start + meta) in one of three layouts:
//   aos   DNode {float4 a, b}: 2 x global_load_dwordx4 per lane (the production layout)
//   soa   8 separate 4-B arrays: 8 x global_load_dword per lane
//   soa2  2 separate float4 arrays (a[], b[]): 2 x dwordx4 from two streams
// and does the slab arithmetic on it. Lanes diverge (random chains), as in traversal; a
// "coherent" run makes all lanes of a wave follow the same chain (the primary-ray top levels).
// build: hipcc --offload-arch=gfx950 -O3 -o layout_bench layout_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

struct alignas(16) Node { float4 a, b; };

__device__ __forceinline__ unsigned next_index(float4 a, float4 b, float ox, float oy, float oz, unsigned n) {
    // slab arithmetic on all six planes (what the box test does with the record), then a
    // data-dependent next index from the record's start/meta words
    const float mx = (a.x - ox) * 1.5f, Mx = (a.y - ox) * 1.5f;
    const float my = (a.z - oy) * 0.5f, My = (a.w - oy) * 0.5f;
    const float mz = (b.x - oz) * 2.5f, Mz = (b.y - oz) * 2.5f;
    const float t0 = fmaxf(fmaxf(fminf(mx, Mx), fminf(my, My)), fminf(mz, Mz));
    const float t1 = fminf(fminf(fmaxf(mx, Mx), fmaxf(my, My)), fmaxf(mz, Mz));
    const unsigned s = __float_as_uint(b.z) ^ (t0 <= t1 ? __float_as_uint(b.w) : 0x9e3779b9u);
    return s % n;
}

template <int L>
__global__ __launch_bounds__(256) void chase(const Node* aos, const float* soa, const float4* sa, const float4* sb,
                                             unsigned n, int steps, int coherent, unsigned* out) {
    const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned idx = (coherent ? (tid >> 6) : tid) * 2654435761u % n;
    const float ox = 0.25f * (threadIdx.x & 7), oy = 0.5f, oz = 0.125f * (threadIdx.x >> 3);
    unsigned acc = 0;
    for (int s = 0; s < steps; s++) {
        float4 a, b;
        if (L == 0) {
            a = aos[idx].a;
            b = aos[idx].b;
        } else if (L == 1) {
            a = make_float4(soa[idx], soa[n + idx], soa[2 * (size_t)n + idx], soa[3 * (size_t)n + idx]);
            b = make_float4(soa[4 * (size_t)n + idx], soa[5 * (size_t)n + idx], soa[6 * (size_t)n + idx], soa[7 * (size_t)n + idx]);
        } else {
            a = sa[idx];
            b = sb[idx];
        }
        idx = next_index(a, b, ox, oy, oz, n);
        acc += idx;
    }
    out[tid] = acc;
}

int main(int argc, char** argv) {
    int cus = 256;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    cus = prop.multiProcessorCount;
    const int blocks = cus * 8, threads = 256, steps = 2000;
    const size_t sizes[] = {240, 1u << 15, 1u << 19, 1u << 22};  // cornellbox-like .. 128 MB of nodes
    const char* names[] = {"aos", "soa", "soa2"};
    printf("device %s, %d CUs; %d lanes x %d dependent node fetches per run\n", prop.name, cus, blocks * threads, steps);
    printf("%-10s %-9s %-5s %10s %14s\n", "nodes", "MB", "layout", "ms", "Gnodes/s");
    for (size_t n : sizes) {
        std::vector<Node> h(n);
        std::vector<float> hs(8 * n);
        std::vector<float4> ha(n), hb(n);
        srand(7);
        for (size_t i = 0; i < n; i++) {
            float v[8];
            for (int k = 0; k < 6; k++) v[k] = (float)rand() / RAND_MAX;
            unsigned st = (unsigned)rand(), me = (unsigned)rand();
            std::memcpy(&v[6], &st, 4);
            std::memcpy(&v[7], &me, 4);
            h[i].a = make_float4(v[0], v[1], v[2], v[3]);
            h[i].b = make_float4(v[4], v[5], v[6], v[7]);
            for (int k = 0; k < 8; k++) hs[k * n + i] = v[k];
            ha[i] = h[i].a;
            hb[i] = h[i].b;
        }
        Node* daos;
        float* dsoa;
        float4 *dsa, *dsb;
        unsigned* dout;
        CHECK(hipMalloc(&daos, n * sizeof(Node)));
        CHECK(hipMalloc(&dsoa, 8 * n * sizeof(float)));
        CHECK(hipMalloc(&dsa, n * sizeof(float4)));
        CHECK(hipMalloc(&dsb, n * sizeof(float4)));
        CHECK(hipMalloc(&dout, (size_t)blocks * threads * 4));
        CHECK(hipMemcpy(daos, h.data(), n * sizeof(Node), hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dsoa, hs.data(), 8 * n * sizeof(float), hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dsa, ha.data(), n * sizeof(float4), hipMemcpyHostToDevice));
        CHECK(hipMemcpy(dsb, hb.data(), n * sizeof(float4), hipMemcpyHostToDevice));
        for (int coherent = 0; coherent < 2; coherent++) {
            std::vector<unsigned> res[3];
            for (int L = 0; L < 3; L++) {
                hipEvent_t e0, e1;
                CHECK(hipEventCreate(&e0));
                CHECK(hipEventCreate(&e1));
                float best = 1e30f;
                for (int rep = 0; rep < 4; rep++) {
                    CHECK(hipEventRecord(e0));
                    if (L == 0) hipLaunchKernelGGL(chase<0>, dim3(blocks), dim3(threads), 0, 0, daos, dsoa, dsa, dsb, (unsigned)n, steps, coherent, dout);
                    if (L == 1) hipLaunchKernelGGL(chase<1>, dim3(blocks), dim3(threads), 0, 0, daos, dsoa, dsa, dsb, (unsigned)n, steps, coherent, dout);
                    if (L == 2) hipLaunchKernelGGL(chase<2>, dim3(blocks), dim3(threads), 0, 0, daos, dsoa, dsa, dsb, (unsigned)n, steps, coherent, dout);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    if (rep > 0 && ms < best) best = ms;
                }
                res[L].resize((size_t)blocks * threads);
                CHECK(hipMemcpy(res[L].data(), dout, res[L].size() * 4, hipMemcpyDeviceToHost));
                printf("%-10zu %-9.2f %-5s %10.3f %14.2f  %s\n", n, n * 32.0 / 1e6, names[L], best,
                       (double)blocks * threads * steps / best / 1e6, coherent ? "coherent" : "divergent");
                CHECK(hipEventDestroy(e0));
                CHECK(hipEventDestroy(e1));
            }
            if (res[0] != res[1] || res[0] != res[2]) {
                printf("layout results differ\n");
                return 1;
            }
        }
        CHECK(hipFree(daos));
        CHECK(hipFree(dsoa));
        CHECK(hipFree(dsa));
        CHECK(hipFree(dsb));
        CHECK(hipFree(dout));
    }
    return 0;
}
