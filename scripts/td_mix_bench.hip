// The vector-memory ceiling for the HBM-mode kernels' own load mix: dependent
// random gathers, as a BVH walk does, of the record shapes the traversal and shading load —
//   mode 0: one 16-B row (dwordx4)                    the round-2 ceiling (td_width_bench mode 0)
//   mode 1: a 64-B wide node record (4 x dwordx4)     node_step_wide
//   mode 2: an 80-B triangle pair (5 x dwordx4)       prim_step
//   mode 3: an 8-B texel pair (dwordx2)               eval_texture
//   mode 4: a 48-B compact wide record (3 x dwordx4)  (candidate: child words packed into row 2)
// over working sets from L2-resident (4 MiB per XCD) through MALL (64-256 MiB) to HBM (2 GiB).
// Every lane walks its own chain (the next record index from the loaded words); all 64 lanes are
// active (td_lanes_bench: the TD charges per wave-instruction, not per active lane). Prints the
// wave-instructions per second per (mode, working set); run it under rocprofv3 --pmc
// TD_TD_BUSY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE to see TD busy and the L2 hit rate of each
// dispatch (one dispatch per line, in print order after a warm-up dispatch).
// usage: td_mix_bench [workgroups per CU (16)] [active lanes per wave (64)]: with fewer than 16
// workgroups each one allocates LDS so that no more fit on a CU (the kernels' residency: 4
// workgroups of 4 waves = 4 waves per SIMD), and only the first `active` lanes of a wave walk.
// build: make -C julia-raytracer_amd td-mix (hipcc --offload-arch=gfx950 -O3)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int MODE>
__global__ __launch_bounds__(256) void chase(const uint4* rec, unsigned n, int steps, unsigned* out, int active) {
    extern __shared__ unsigned pad[];  // sized by the launch only to cap workgroups per CU
    if ((int)(threadIdx.x & 63) >= active) return;
    if (steps < 0) pad[threadIdx.x] = 0;  // never: keeps the allocation
    unsigned i = ((blockIdx.x * 256u + threadIdx.x) * 2654435761u) & (n - 1);  // n: a power of two
    unsigned acc = 0;
    for (int s = 0; s < steps; s++) {
        unsigned v;
        if (MODE == 0) {
            const uint4 a = rec[(size_t)i];
            v = a.x ^ a.y ^ a.z ^ a.w;
        } else if (MODE == 1) {
            const uint4* r = rec + 4 * (size_t)i;
            const uint4 a = r[0], b = r[1], c = r[2], d = r[3];
            v = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
        } else if (MODE == 2) {
            const uint4* r = rec + 5 * (size_t)i;
            const uint4 a = r[0], b = r[1], c = r[2], d = r[3], e = r[4];
            v = a.x ^ b.y ^ c.z ^ d.w ^ e.x ^ a.w ^ b.x ^ c.y ^ d.z ^ e.w;
        } else if (MODE == 4) {
            const uint4* r = rec + 3 * (size_t)i;
            const uint4 a = r[0], b = r[1], c = r[2];
            v = a.x ^ b.y ^ c.z ^ a.w ^ b.x ^ c.y;
        } else {
            const uint2 a = reinterpret_cast<const uint2*>(rec)[(size_t)i];
            v = a.x ^ a.y;
        }
        acc += v;
        i = (v * 2654435761u + (unsigned)s) & (n - 1);
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

template <int MODE>
float run(const uint4* rec, unsigned n, unsigned* out, int blocks, int steps, int active, size_t lds) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    chase<MODE><<<blocks, 256, lds>>>(rec, n, steps, out, active);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms;
}

__global__ void fill(uint4* p, size_t n16) {
    for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < n16; k += (size_t)gridDim.x * 256) {
        unsigned x = (unsigned)k * 2654435761u + 12345u;
        p[k] = make_uint4(x, x * 1664525u + 1013904223u, x ^ 0x9e3779b9u, x * 22695477u + 1u);
    }
}

int main(int argc, char** argv) {
    const size_t max_bytes = 2ull << 30;  // 2 GiB: the HBM working set
    uint4* rec;
    unsigned* out;
    const int per_cu = argc > 1 ? atoi(argv[1]) : 16;  // 16 workgroups (64 waves) per CU: every SIMD's wave slots filled
    const int active = argc > 2 ? atoi(argv[2]) : 64;
    const int blocks = 256 * per_cu;
    // fewer workgroups per CU: each takes a 1/per_cu share of the CU's 160 KiB of LDS
    const size_t lds = per_cu < 16 ? (160u << 10) / (unsigned)per_cu - 1024 : 0;
    if (lds > 0) (void)hipFuncSetAttribute((const void*)chase<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                 (void)hipFuncSetAttribute((const void*)chase<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                 (void)hipFuncSetAttribute((const void*)chase<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                 (void)hipFuncSetAttribute((const void*)chase<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                 (void)hipFuncSetAttribute((const void*)chase<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    printf("workgroups per CU %d (LDS %zu B each), active lanes per wave %d\n", per_cu, lds, active);
    if (hipMalloc(&rec, max_bytes) != hipSuccess || hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    fill<<<4096, 256>>>(rec, max_bytes / 16);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const size_t sets[4] = {4ull << 20, 64ull << 20, 256ull << 20, 2ull << 30};
    const char* name[5] = {"16 B row (dwordx4)", "64 B wide node (4 x dwordx4)", "80 B tri pair (5 x dwordx4)",
                           "8 B texel pair (dwordx2)", "48 B compact wide (3 x dwordx4)"};
    const int insts[5] = {1, 4, 5, 1, 3};
    const int rec_bytes[5] = {16, 64, 80, 8, 48};
    run<0>(rec, 1u << 16, out, blocks, 200, active, lds);  // warm-up dispatch
    for (int m = 0; m < 5; m++) {
        for (int w = 0; w < 4; w++) {
            unsigned n = 1;
            while ((size_t)(n * 2ull) * rec_bytes[m] <= sets[w]) n *= 2;
            const int steps = m == 0 || m == 3 ? 20000 : 5000;
            float ms = m == 0 ? run<0>(rec, n, out, blocks, steps, active, lds)
                     : m == 1 ? run<1>(rec, n, out, blocks, steps, active, lds)
                     : m == 2 ? run<2>(rec, n, out, blocks, steps, active, lds)
                     : m == 3 ? run<3>(rec, n, out, blocks, steps, active, lds)
                              : run<4>(rec, n, out, blocks, steps, active, lds);
            const double waves = (double)blocks * 4 * steps;  // 4 waves per workgroup
            printf("mode %d %-30s set %5zu MiB  %8.2f ms  %8.2f G wave-instr/s  %8.1f G records/s\n", m, name[m],
                   ((size_t)n * rec_bytes[m]) >> 20, ms, waves * insts[m] / ms * 1e-6,
                   waves * active / ms * 1e-6);
        }
    }
    return 0;
}
