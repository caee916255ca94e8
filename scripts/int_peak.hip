// Microbenchmark: issue cost of the integer ops of the PCG32 step on gfx950 (v_mul_lo_u32,
// v_mad_u64_u32, v_add_u32, v_alignbit_b32, v_cvt_f32_u32), 8 independent chains per lane,
// every operand in VGPRs, 8 waves per SIMD. Prints cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned *out, int iters, unsigned m_arg)
{
    unsigned m = m_arg + (threadIdx.x & 1);
    asm volatile("" : "+v"(m));
    unsigned a[8];
    unsigned long long b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = threadIdx.x + j; b[j] = threadIdx.x * 7ull + j; }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (OP == 0) a[j] = a[j] * m;                                   // v_mul_lo_u32
                if (OP == 1) b[j] = (unsigned long long)(unsigned)b[j] * m + b[j]; // v_mad_u64_u32
                if (OP == 2) a[j] = a[j] + m;                                   // v_add_u32
                if (OP == 3) a[j] = __builtin_amdgcn_alignbit(a[j], m, a[j] & 31); // v_alignbit_b32
                if (OP == 4) a[j] = __float_as_uint((float)a[j]);               // v_cvt_f32_u32
                if (OP == 5) a[j] = __umul24(a[j], m);                          // v_mul_u32_u24
                if (OP == 1) asm volatile("" : "+v"(b[j]));
                else asm volatile("" : "+v"(a[j]));
            }
    }
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + (unsigned)b[j] + (unsigned)(b[j] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP> int run(const char *name, unsigned *d, int cus)
{
    const int iters = 2000, grid = cus * 8;  // 8 WG of 256 per CU = 8 waves per SIMD
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, d, 10, 0x4C957F2Du);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(256), 0, 0, d, iters, 0x4C957F2Du);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double instr = (double)grid * 4 * iters * 64;  // wave-instructions (4 waves per WG, 64 per iter)
    const double per_simd = instr / (cus * 4);
    printf("%-28s %8.3f ms  %.2f cyc/wave-instr/SIMD @2.4GHz\n", name, ms, ms * 1e-3 * 2.4e9 / per_simd);
    return 0;
}

int main()
{
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned *d;
    CHECK(hipMalloc(&d, (size_t)cus * 8 * 256 * 4));
    run<2>("v_add_u32", d, cus);
    run<0>("v_mul_lo_u32", d, cus);
    run<1>("v_mad_u64_u32 (+64-bit add)", d, cus);
    run<3>("v_alignbit_b32", d, cus);
    run<4>("v_cvt_f32_u32", d, cus);
    run<5>("v_mul_u32_u24", d, cus);
    return 0;
}
