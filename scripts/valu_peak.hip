// Microbenchmark: sustained VALU issue rate on gfx950 for the instruction shapes of the
// render loop (independent f32 add/mul/fma, packed f32, LDS-broadcast-fed loop). Prints
// cycles per wave-instruction per SIMD at the measured clock, and TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <utility>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k(float *out, int iters, float s_arg)
{
    // OP >= 10: same op with every operand in VGPRs (s made lane-varying, opaque to the compiler)
    float s = s_arg;
    if (OP >= 10) { s = s_arg + (float)(threadIdx.x & 1) * 1e-30f; asm volatile("" : "+v"(s)); }
    float one = 1.f;
    if (OP >= 10) asm volatile("" : "+v"(one));
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP % 10 == 0) { a0 = fmaf(a0, s, one); a1 = fmaf(a1, s, one); a2 = fmaf(a2, s, one); a3 = fmaf(a3, s, one);
                           a4 = fmaf(a4, s, one); a5 = fmaf(a5, s, one); a6 = fmaf(a6, s, one); a7 = fmaf(a7, s, one); }
            if (OP % 10 == 1) { a0 = a0 + s; a1 = a1 + s; a2 = a2 + s; a3 = a3 + s; a4 = a4 + s; a5 = a5 + s; a6 = a6 + s; a7 = a7 + s; }
            if (OP % 10 == 2) { a0 = a0 * s; a1 = a1 * s; a2 = a2 * s; a3 = a3 * s; a4 = a4 * s; a5 = a5 * s; a6 = a6 * s; a7 = a7 * s; }
            if (OP % 10 == 3) { // packed: 4 v_pk_fma_f32 per 8 values
                typedef float f2 __attribute__((ext_vector_type(2)));
                f2 x0 = {a0, a1}, x1 = {a2, a3}, x2 = {a4, a5}, x3 = {a6, a7}, ss = {s, s}, o2 = {one, one};
                x0 = __builtin_elementwise_fma(x0, ss, o2); x1 = __builtin_elementwise_fma(x1, ss, o2);
                x2 = __builtin_elementwise_fma(x2, ss, o2); x3 = __builtin_elementwise_fma(x3, ss, o2);
                a0 = x0.x; a1 = x0.y; a2 = x1.x; a3 = x1.y; a4 = x2.x; a5 = x2.y; a6 = x3.x; a7 = x3.y; }
            if (OP % 10 == 4) { a0 = fmaf(a0, s, one); a0 = fmaf(a0, s, one); a0 = fmaf(a0, s, one); a0 = fmaf(a0, s, one);
                           a0 = fmaf(a0, s, one); a0 = fmaf(a0, s, one); a0 = fmaf(a0, s, one); a0 = fmaf(a0, s, one); }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// The render loop's shape: 17 exact ops (FAST: 11 with FMA) per sphere, spheres either
// broadcast from LDS (ds_read_b128 per sphere) or held 16-per-row in VGPRs and fed through
// DPP row_newbcast operands (one ds_read_b128 per 16 spheres).
template <int K> __device__ __forceinline__ float bc(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x150 + K, 0xf, 0xf, false));
}
template <bool FAST>
__device__ __forceinline__ float test(float cx, float cy, float cz, float rr, float ox, float oy, float oz, float dx,
                                      float dy, float dz, float a)
{
    const float ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    if (FAST) {
        const float b = fmaf(ocx, dx, fmaf(ocy, dy, ocz * dz));
        const float c = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -rr)));
        return fmaf(b, b, -(a * c));
    }
    const float b = ocx * dx + ocy * dy + ocz * dz;
    const float c = ocx * ocx + ocy * ocy + ocz * ocz - rr;
    return b * b - a * c;
}
template <bool FAST, int... K>
__device__ __forceinline__ void dpp16(std::integer_sequence<int, K...>, float4 s, float ox, float oy, float oz, float dx,
                                      float dy, float dz, float a, float &m)
{
    float dq[sizeof...(K)] = {test<FAST>(bc<K>(s.x), bc<K>(s.y), bc<K>(s.z), bc<K>(s.w), ox, oy, oz, dx, dy, dz, a)...};
#pragma unroll
    for (int k = 0; k < (int)sizeof...(K); k += 8)
        m = fmaxf(m, fmaxf(fmaxf(fmaxf(dq[k], dq[k + 1]), fmaxf(dq[k + 2], dq[k + 3])),
                           fmaxf(fmaxf(dq[k + 4], dq[k + 5]), fmaxf(dq[k + 6], dq[k + 7]))));
}
template <bool DPP, bool FAST>
__global__ __launch_bounds__(256) void sph(float *out, int iters, const float4 *g, int n)
{
    extern __shared__ float4 L[];
    for (int i = threadIdx.x; i < n; i += 256) L[i] = g[i];
    __syncthreads();
    float ox = threadIdx.x * 1e-3f, oy = 1.f + threadIdx.x * 2e-4f, oz = 2.f - threadIdx.x * 1e-4f;
    float dx = .3f + threadIdx.x * 1e-5f, dy = -.2f, dz = .9f;
    asm volatile("" : "+v"(dy), "+v"(dz));
    float a = dx * dx + dy * dy + dz * dz, acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        float m = -1.f;
        if (DPP) {
            for (int i = 0; i < n; i += 16) {
                const float4 s = L[i + (threadIdx.x & 15)];
                dpp16<FAST>(std::make_integer_sequence<int, 16>{}, s, ox, oy, oz, dx, dy, dz, a, m);
            }
        } else {
            for (int i = 0; i < n; i += 8) {
                float dq[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float4 s = L[i + k];
                    dq[k] = test<FAST>(s.x, s.y, s.z, s.w, ox, oy, oz, dx, dy, dz, a);
                }
                m = fmaxf(m, fmaxf(fmaxf(fmaxf(dq[0], dq[1]), fmaxf(dq[2], dq[3])), fmaxf(fmaxf(dq[4], dq[5]), fmaxf(dq[6], dq[7]))));
            }
        }
        acc += m;
        ox += 1e-6f;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main()
{
    hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    float *out; CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4 * 4));
    hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    const char *names[] = {"v_fma_f32 x8 indep", "v_add_f32 x8 indep", "v_mul_f32 x8 indep", "v_pk_fma_f32 x4 (8 fma)", "v_fma_f32 dep chain"};
    for (int wg_per_cu : {8}) {
        for (int opi = 5; opi < 10; ++opi) {
            const int op = opi % 5, vg = opi >= 5;
            const int iters = 20000;
            auto launch = [&]() {
                dim3 g(cus * wg_per_cu), b(256);
                switch (op + 10 * vg) {
                case 0: hipLaunchKernelGGL(k<0>, g, b, 0, 0, out, iters, 0.999f); break;
                case 1: hipLaunchKernelGGL(k<1>, g, b, 0, 0, out, iters, 0.999f); break;
                case 2: hipLaunchKernelGGL(k<2>, g, b, 0, 0, out, iters, 0.999f); break;
                case 3: hipLaunchKernelGGL(k<3>, g, b, 0, 0, out, iters, 0.999f); break;
                case 4: hipLaunchKernelGGL(k<4>, g, b, 0, 0, out, iters, 0.999f); break;
                case 10: hipLaunchKernelGGL(k<10>, g, b, 0, 0, out, iters, 0.999f); break;
                case 11: hipLaunchKernelGGL(k<11>, g, b, 0, 0, out, iters, 0.999f); break;
                case 12: hipLaunchKernelGGL(k<12>, g, b, 0, 0, out, iters, 0.999f); break;
                case 13: hipLaunchKernelGGL(k<13>, g, b, 0, 0, out, iters, 0.999f); break;
                case 14: hipLaunchKernelGGL(k<14>, g, b, 0, 0, out, iters, 0.999f); break;
                }
            };
            launch(); CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0)); launch(); CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double waves = (double)cus * wg_per_cu * 4;
            const double instrs = waves * iters * (op == 3 ? 32 : 64);      // wave-instructions
            const double flop = (double)cus * wg_per_cu * 256 * iters * 64 * (op == 1 || op == 2 ? 1 : 2) * (op == 4 ? 1.0 / 8 * 8 : 1);
            const double per_simd = instrs / (cus * 4.0);
            printf("%s wg/cu=%d waves/simd=%d %-26s %.3f ms  %.2f ns/instr/SIMD  (%.2f cyc @2.4GHz)  %.1f TFLOP/s\n", vg ? "VGPR-only" : "SGPR-operand", wg_per_cu,
                   wg_per_cu, names[op], ms, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4, flop / ms / 1e9);
        }
    }
    // sphere-loop shapes
    std::vector<float4> h(496);
    for (int i = 0; i < 496; ++i) h[i] = make_float4(i * .01f, .2f, -i * .01f, .04f);
    float4 *g; CHECK(hipMalloc(&g, 496 * 16)); CHECK(hipMemcpy(g, h.data(), 496 * 16, hipMemcpyHostToDevice));
    const char *sn[] = {"LDS exact", "DPP exact", "LDS fast ", "DPP fast "};
    for (int v = 0; v < 4; ++v) {
        for (int wg_per_cu : {4, 7, 8}) {
            const int iters = 200;
            dim3 gr(cus * wg_per_cu), b(256);
            auto go = [&]() {
                switch (v) {
                case 0: hipLaunchKernelGGL((sph<false, false>), gr, b, 496 * 16, 0, out, iters, g, 496); break;
                case 1: hipLaunchKernelGGL((sph<true, false>), gr, b, 496 * 16, 0, out, iters, g, 496); break;
                case 2: hipLaunchKernelGGL((sph<false, true>), gr, b, 496 * 16, 0, out, iters, g, 496); break;
                case 3: hipLaunchKernelGGL((sph<true, true>), gr, b, 496 * 16, 0, out, iters, g, 496); break;
                }
            };
            go(); CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0)); go(); CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double tests = (double)cus * wg_per_cu * 256 * iters * 496;
            printf("sphere loop %s wg/cu=%d: %.3f ms  %.3f Ttests/s  -> %.1f TFLOP/s at 20 FLOP/test\n", sn[v], wg_per_cu, ms,
                   tests / ms / 1e9, tests * 20 / ms / 1e9);
        }
    }
    return 0;
}
