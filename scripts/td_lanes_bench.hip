// Vector-memory gather cost by ACTIVE LANES per wave on gfx950. The HBM-mode traversal kernels
// are TD-bound (TD busy 98 %) while their loads run with few lanes active (traversal lane
// utilisation ~0.2). Is a gather wave-instruction charged per instruction or per active lane?
// Every active lane chases dependent 16-B gathers (one dwordx4, a BVH pop's start/meta load) over
// an array of 32-B records; lanes >= K of each wave skip the loop. Array sizes: 4 MiB (L2-resident
// per XCD) and 64 MiB (beyond L2, in the 256 MiB MALL). C independent chains per lane (C = 1:
// latency-bound; C = 4, 8: enough loads in flight to expose the return path's throughput).
// Prints G wave-instructions/s and G lane-loads/s per (C, K).
// build: hipcc --offload-arch=gfx950 -O3 -o build/td_lanes_bench scripts/td_lanes_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int C>
__global__ __launch_bounds__(256) void chase(const uint4* rec, unsigned n, int steps, int k, unsigned* out) {
    const unsigned lane = threadIdx.x & 63;
    unsigned i[C];
    for (int c = 0; c < C; c++)  // n: a power of two
        i[c] = ((blockIdx.x * 256u + threadIdx.x) * 2654435761u + 40503u * (unsigned)c) & (n - 1);
    unsigned acc = 0;
    if (lane < (unsigned)k) {
        for (int s = 0; s < steps; s++) {
#pragma unroll
            for (int c = 0; c < C; c++) {
                const uint4 a = rec[2 * (size_t)i[c]];
                const unsigned v = a.x ^ a.y ^ a.z ^ a.w;
                acc += v;
                i[c] = (v * 2654435761u + (unsigned)s) & (n - 1);
            }
        }
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

template <int C>
float run(const uint4* rec, unsigned n, int steps, int k, unsigned* out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    chase<C><<<blocks, 256>>>(rec, n, steps, k, out);
    hipEventRecord(a);
    chase<C><<<blocks, 256>>>(rec, n, steps, k, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms;
}

int main() {
    const unsigned sizes[2] = {1u << 17, 1u << 21};  // records of 32 B: 4 MiB, 64 MiB
    const int ks[7] = {64, 48, 32, 16, 8, 4, 1};
    const int blocks = 256 * 16, steps = 2000;
    unsigned* out;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    for (unsigned n : sizes) {
        std::vector<uint4> h(2 * (size_t)n);
        unsigned x = 12345;
        for (auto& r : h) {
            x = x * 1664525u + 1013904223u; r.x = x;
            x = x * 1664525u + 1013904223u; r.y = x;
            x = x * 1664525u + 1013904223u; r.z = x;
            x = x * 1664525u + 1013904223u; r.w = x;
        }
        uint4* rec;
        if (hipMalloc(&rec, h.size() * 16) != hipSuccess) return 1;
        hipMemcpy(rec, h.data(), h.size() * 16, hipMemcpyHostToDevice);
        for (int c : {1, 4, 8})
            for (int k : ks) {
                const float ms = c == 1 ? run<1>(rec, n, steps, k, out, blocks)
                                 : c == 4 ? run<4>(rec, n, steps, k, out, blocks) : run<8>(rec, n, steps, k, out, blocks);
                const double insts = (double)blocks * 4 * steps * c;
                printf("array %3u MiB  chains %d  active lanes %2d  %8.2f ms  %7.2f G wave-instr/s  %7.1f G lane-loads/s\n",
                       (unsigned)(n * 32ull >> 20), c, k, ms, insts / ms * 1e-6, insts * k / ms * 1e-6);
            }
        hipFree(rec);
    }
    return 0;
}
