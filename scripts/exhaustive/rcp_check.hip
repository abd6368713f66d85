// Exhaustive check (all 2^32 float bit patterns) that a reciprocal built from v_rcp_f32 and FMA
// Newton corrections equals the IEEE-correct 1.0f / x the kernel uses today (-ffp-contract=off,
// no fast math). Prints the mismatch counts per variant and the first few mismatching inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float rcp1(float x) {  // one Newton step
    float r = __builtin_amdgcn_rcpf(x);
    float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float rcp2(float x) {  // two Newton steps
    float r = rcp1(x);
    float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ bool same(float a, float b) {
    unsigned ua = __float_as_uint(a), ub = __float_as_uint(b);
    return ua == ub || (a != a && b != b);
}
__global__ void check(unsigned long long base, unsigned long long* bad, unsigned* first) {
    unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    float x = __uint_as_float((unsigned)i);
    volatile float one = 1.0f;
    float ref = one / x;
    if (!same(rcp1(x), ref)) {
        unsigned long long n = atomicAdd(bad + 0, 1ull);
        if (n < 8) first[n] = (unsigned)i;
    }
    if (!same(rcp2(x), ref)) {
        unsigned long long n = atomicAdd(bad + 1, 1ull);
        if (n < 8) first[8 + n] = (unsigned)i;
    }
}
int main() {
    unsigned long long* bad;
    unsigned* first;
    hipMalloc(&bad, 16);
    hipMalloc(&first, 64);
    hipMemset(bad, 0, 16);
    hipMemset(first, 0, 64);
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, b, bad, first);
    unsigned long long h[2];
    unsigned f[16];
    hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
    printf("one-step mismatches: %llu\ntwo-step mismatches: %llu\n", h[0], h[1]);
    for (int k = 0; k < 8 && k < (int)h[0]; k++) { float v; memcpy(&v, &f[k], 4); printf("  1-step bad x=%08x (%g)\n", f[k], v); }
    for (int k = 0; k < 8 && k < (int)h[1]; k++) { float v; memcpy(&v, &f[8 + k], 4); printf("  2-step bad x=%08x (%g)\n", f[8 + k], v); }
    return 0;
}
