// Vector-memory return cost by load width on gfx950: is the TD (texture data) path, which binds
// the HBM-mode traversal kernels (TD busy 95-99 %), charged per byte or per wave-instruction?
// Every lane chases dependent gathers over an L2-resident array of 32-B records (one random
// record per step, the next index from the loaded words, as a BVH pop does) and loads
//   mode 0: 16 B (one dwordx4)        mode 1: 24 B (dwordx4 + dwordx2)
//   mode 2: 32 B (two dwordx4)        mode 3: 8 B (one dwordx2)      mode 4: 4 B (one dword)
// per step. Prints G records/s and G load instructions/s per mode.
// build: hipcc --offload-arch=gfx950 -O3 -o build/td_width_bench scripts/td_width_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(256) void chase(const uint4* rec, unsigned n, int steps, unsigned* out) {
    unsigned i = ((blockIdx.x * 256u + threadIdx.x) * 2654435761u) & (n - 1);  // n: a power of two
    unsigned acc = 0;
    for (int s = 0; s < steps; s++) {
        const uint4* r = rec + 2 * (size_t)i;
        unsigned v;
        if (MODE == 0) {
            const uint4 a = r[0];
            v = a.x ^ a.y ^ a.z ^ a.w;
        } else if (MODE == 1) {
            const uint4 a = r[0];
            const uint2 b = *reinterpret_cast<const uint2*>(r + 1);
            v = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y;
        } else if (MODE == 2) {
            const uint4 a = r[0], b = r[1];
            v = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        } else if (MODE == 3) {
            const uint2 a = *reinterpret_cast<const uint2*>(r);
            v = a.x ^ a.y;
        } else {
            v = *reinterpret_cast<const unsigned*>(r);
        }
        acc += v;
        i = (v * 2654435761u + (unsigned)s) & (n - 1);
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

template <int MODE>
double run(const uint4* rec, unsigned n, unsigned* out, int blocks, int steps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    chase<MODE><<<blocks, 256>>>(rec, n, steps, out);
    hipEventRecord(a);
    chase<MODE><<<blocks, 256>>>(rec, n, steps, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const unsigned n = 1u << 17;  // 131072 records x 32 B = 4 MiB: L2-resident per XCD
    std::vector<uint4> h(2 * (size_t)n);
    unsigned x = 12345;
    for (auto& r : h) {
        x = x * 1664525u + 1013904223u; r.x = x;
        x = x * 1664525u + 1013904223u; r.y = x;
        x = x * 1664525u + 1013904223u; r.z = x;
        x = x * 1664525u + 1013904223u; r.w = x;
    }
    uint4* rec;
    unsigned* out;
    const int blocks = 256 * 16, steps = 2000;
    if (hipMalloc(&rec, h.size() * 16) != hipSuccess || hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    hipMemcpy(rec, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    const double lanes = (double)blocks * 256 * steps;
    const char* name[5] = {"16 B: dwordx4", "24 B: dwordx4 + dwordx2", "32 B: 2 x dwordx4", "8 B: dwordx2", "4 B: dword"};
    const int insts[5] = {1, 2, 2, 1, 1};
    double ms[5] = {run<0>(rec, n, out, blocks, steps), run<1>(rec, n, out, blocks, steps),
                    run<2>(rec, n, out, blocks, steps), run<3>(rec, n, out, blocks, steps),
                    run<4>(rec, n, out, blocks, steps)};
    for (int m = 0; m < 5; m++)
        printf("mode %d %-26s %8.2f ms  %7.1f G records/s  %7.1f G lane-loads/s\n", m, name[m], ms[m],
               lanes / ms[m] * 1e-6, lanes * insts[m] / ms[m] * 1e-6);
    return 0;
}
