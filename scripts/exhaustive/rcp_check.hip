// Exhaustive check over all 2^32 float bit patterns that jl_rcp (julia-raytracer_amd/csrc/
// jt_device.h: v_rcp_f32 + one FMA Newton step in the normal range, IEEE division elsewhere)
// equals the IEEE-correct 1.0f / x, bit for bit (NaNs compare equal). Also reports the bare
// one-step formula, whose mismatches are exactly the inputs routed to the division.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../julia-raytracer_amd/csrc -o rcp_check rcp_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#include "jt_device.h"

__device__ __forceinline__ float rcp1(float x) {
    float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
}
__device__ __forceinline__ bool same(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}
__global__ void check(unsigned long long base, unsigned long long* bad, unsigned* first) {
    unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    float x = __uint_as_float((unsigned)i);
    volatile float one = 1.0f;
    float ref = one / x;
    if (!same(jtd::jl_rcp(x), ref)) {
        unsigned long long n = atomicAdd(bad + 0, 1ull);
        if (n < 8) first[n] = (unsigned)i;
    }
    if (!same(rcp1(x), ref)) {
        unsigned long long n = atomicAdd(bad + 1, 1ull);
        if (n < 8) first[8 + n] = (unsigned)i;
    }
}
int main() {
    unsigned long long* bad;
    unsigned* first;
    if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&first, 64) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 16);
    (void)hipMemset(first, 0, 64);
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, b, bad, first);
    unsigned long long h[2];
    unsigned f[16];
    if (hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(f, first, 64, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    printf("jl_rcp mismatches over 2^32 inputs: %llu\nbare one-step formula mismatches: %llu\n", h[0], h[1]);
    for (int k = 0; k < 8 && k < (int)h[0]; k++) printf("  jl_rcp bad x=%08x\n", f[k]);
    return h[0] == 0 ? 0 : 1;
}
