// Exhaustive check of an exact float decision of the slab test's final compare (slab_fast
// below; measured slower than the double compare on gfx950 and not adopted)
// against the reference's Float64 compare
// `t0 <= Float64(t1) * 1.00000024` (src/geometry.jl:102-103), for EVERY float t1 (2^32 bit
// patterns) and, for each, every t0 in the window where the two could disagree: the 24 floats
// from 4 ulps below t1 to 20 ulps above it, and the 8 floats around RN_f(t1 * k), plus t0 = tmin
// and t0 = +inf. The kernel's precondition holds throughout: t0 >= tmin = 1e-4 (t0 is a max
// with ray_eps) and t0 is not NaN (NaN slabs are culled before the compare).
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o slab_check slab_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>

// Decided in float where that is exact; callers guarantee t0 >= tmin > 0 (t0 is a max with
// ray_eps) for non-NaN slabs. t0 <= t1 implies t0 <= t1*c (c > 1, t1 > 0). t0 > RN_f(t1 * k),
// k = 1 + 5*2^-23, implies t0 > RN_d(t1*c), since k(1 - 2^-24) > c(1 + 2^-53) for t1 > 0 (a
// denormal, zero or negative t1 is below tmin either way). Only t1 < t0 <= RN_f(t1 k), a few
// ulps, takes the double compare, behind a wave-uniform branch.
__device__ __forceinline__ bool slab_fast(float t0, float t1) {
    bool pass = t0 <= t1;
    const bool amb = !pass && t0 <= t1 * 1.0000006f;
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(amb) != 0, 0)) {
        if (amb) pass = (double)t0 <= (double)t1 * 1.00000024;
    }
    return pass;
}

__device__ __forceinline__ void one(float t0, float t1, unsigned long long* bad, unsigned* first) {
    if (!(t0 >= 1e-4f)) return;  // precondition (also drops NaN t0)
    const bool fast = slab_fast(t0, t1);
    const bool ref = (double)t0 <= (double)t1 * 1.00000024;
    if (fast != ref) {
        unsigned long long n = atomicAdd(bad, 1ull);
        if (n < 8) {
            first[2 * n] = __float_as_uint(t0);
            first[2 * n + 1] = __float_as_uint(t1);
        }
    }
}
__global__ void check(unsigned long long base, unsigned long long* bad, unsigned* first,
                      unsigned long long* tested) {
    const unsigned b1 = (unsigned)(base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x);
    const float t1 = __uint_as_float(b1);
    unsigned n = 0;
    for (int d = -4; d < 20; d++) {
        one(__uint_as_float(b1 + (unsigned)d), t1, bad, first);
        n++;
    }
    const unsigned bk = __float_as_uint(t1 * 1.0000006f);
    for (int d = -4; d < 4; d++) {
        one(__uint_as_float(bk + (unsigned)d), t1, bad, first);
        n++;
    }
    one(1e-4f, t1, bad, first);
    one(__builtin_inff(), t1, bad, first);
    n += 2;
    if ((threadIdx.x & 63) == 0) atomicAdd(tested, 64ull * n);
}
int main() {
    unsigned long long *bad, *tested;
    unsigned* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&tested, 8) != hipSuccess || hipMalloc(&first, 64) != hipSuccess)
        return 2;
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(tested, 0, 8);
    (void)hipMemset(first, 0, 64);
    const unsigned long long chunk = 1ull << 28;
    for (unsigned long long b = 0; b < (1ull << 32); b += chunk)
        hipLaunchKernelGGL(check, dim3(chunk / 256), dim3(256), 0, 0, b, bad, first, tested);
    unsigned long long h = 0, t = 0;
    unsigned f[16];
    if (hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(&t, tested, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(f, first, 64, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    printf("slab_fast vs the Float64 compare: %llu (t0, t1) pairs generated over all 2^32 t1, "
           "%llu mismatches\n", t, h);
    for (int k = 0; k < 8 && k < (int)h; k++) printf("  bad t0=%08x t1=%08x\n", f[2 * k], f[2 * k + 1]);
    return h == 0 ? 0 : 1;
}
