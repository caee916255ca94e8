// Exhaustive check of sqrt_scaled (rt_kernel.hip: the compiler's IEEE sqrt expansion — hardware
// v_sqrt_f32, then the one-ulp neighbours tested by FMA residuals — on x * 2^32, scaled back) for
// every binary32 x in (0, 2^96): that it is the correctly rounded root, and how often gfx950's
// hardware result already is that root, one ulp below, or one ulp above it (a neighbour that
// never occurs needs no test).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/sqrt_check.hip -o scripts/_bin_sqrt_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

// sqrt_scaled of rt_kernel.hip: the expansion run on x * 2^32 and scaled back by 2^-16
__device__ float sqrt_scaled(float x, int &d)
{
    const float xs = x * 0x1p32f;
    const float s = __builtin_amdgcn_sqrtf(xs);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
    const float sup = __uint_as_float(__float_as_uint(s) + 1u);
    float r = fmaf(-sdn, s, xs) <= 0.f ? sdn : s;
    r = fmaf(-sup, s, xs) > 0.f ? sup : r;
    d = (int)(__float_as_uint(s) - __float_as_uint(r));  // hardware result against the corrected one
    return r * 0x1p-16f;
}

// every positive x below 2^96 (denormals included): counts [0] hardware exact, [1] one ulp below,
// [2] one ulp above, [3] other, [4] sqrt_scaled != the correctly rounded root
__global__ void check(unsigned long long *cnt, uint32_t base)
{
    const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = bits >= 1u && bits < 0x6f800000u;  // (0, 2^96)
    const float x = __uint_as_float(in ? bits : 0x3f800000u);
    int d;
    const float r = sqrt_scaled(x, d);
    // (float)sqrt((double)x) is correctly rounded (53 >= 2 * 24 + 2: no double-rounding error)
    const float rd = (float)sqrt((double)x);
    const bool c[5] = {in && d == 0, in && d == -1, in && d == 1, in && (d < -1 || d > 1),
                       in && __float_as_uint(rd) != __float_as_uint(r)};
    for (int k = 0; k < 5; ++k) {
        const uint64_t m = __ballot(c[k]);
        if ((threadIdx.x & 63u) == 0 && m) atomicAdd(&cnt[k], (unsigned long long)__popcll(m));
    }
}

int main()
{
    unsigned long long *cnt;
    (void)hipMalloc(&cnt, 5 * sizeof(unsigned long long));
    (void)hipMemset(cnt, 0, 5 * sizeof(unsigned long long));
    const uint32_t chunk = 1u << 28;
    for (uint64_t base = 0; base < (1ull << 31); base += chunk)
        check<<<chunk / 256, 256>>>(cnt, (uint32_t)base);
    unsigned long long h[5];
    (void)hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost);
    printf("x in (0, 2^96): hw exact %llu, hw one ulp below %llu, hw one ulp above %llu, other %llu; "
           "sqrt_scaled != correctly rounded: %llu\n", h[0], h[1], h[2], h[3], h[4]);
    (void)hipFree(cnt);
    return 0;
}
