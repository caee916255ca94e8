// Issue-cost probe for the instruction shapes of render_kernel's hot loop on gfx950: operand
// kinds (VGPR, SGPR, literal, inline constant), integer ops of the PCG32 step, compares and
// selects with VCC or an SGPR-pair mask, DPP, f64. 8 independent chains per lane, 8 waves per
// SIMD; prints cycles per wave-instruction per SIMD at the reported clock.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_int.hip -o scripts/_bin_ubench_int
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <utility>
#include <cstdlib>

constexpr int kIters = 16384;

#define C8(stmt) \
    {            \
        stmt(0); \
        stmt(1); \
        stmt(2); \
        stmt(3); \
        stmt(4); \
        stmt(5); \
        stmt(6); \
        stmt(7); \
    }

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t *out, uint32_t c)
{
    uint32_t x[8];
    uint64_t y[8];
    uint32_t v = c + (threadIdx.x & 1);  // lane-varying operand in a VGPR
    asm volatile("" : "+v"(v));
    for (int i = 0; i < 8; ++i) {
        x[i] = threadIdx.x * 7u + i * 77u;
        y[i] = x[i] * 3ull;
    }
    uint64_t m = 0;
    asm volatile("s_mov_b64 %0, exec" : "=s"(m));
    for (int it = 0; it < kIters; ++it) {
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(x[i]) : "v"(v))
        if (OP == 0) C8(X)
#undef X
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(x[i]) : "s"(c))
        if (OP == 1) C8(X)
#undef X
#define X(i) asm volatile("v_mul_f32 %0, 0x3f800001, %0" : "+v"(x[i]))
        if (OP == 2) C8(X)
#undef X
#define X(i) asm volatile("v_fma_f32 %0, %0, 2.0, %0" : "+v"(x[i]))
        if (OP == 3) C8(X)
#undef X
#define X(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(v) : "vcc")
        if (OP == 4) C8(X)
#undef X
#define X(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[i]) : "v"(v), "s"(m))
        if (OP == 5) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_lt_f32 vcc, %0, %1" ::"v"(x[i]), "v"(v) : "vcc")
        if (OP == 6) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x[i]), "v"(v))
        if (OP == 7) C8(X)
#undef X
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 8) C8(X)
#undef X
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 9) C8(X)
#undef X
#define X(i) asm volatile("v_mad_u64_u32 %0, %3, %1, %2, %0" : "+v"(y[i]) : "v"(x[i]), "v"(v), "s"(m))
        if (OP == 10) C8(X)
#undef X
#define X(i) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 11) C8(X)
#undef X
#define X(i) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x[i]))
        if (OP == 12) C8(X)
#undef X
#define X(i) asm volatile("v_min_f32 %0, 0x4f7fffff, %0" : "+v"(x[i]))
        if (OP == 13) C8(X)
#undef X
#define X(i) asm volatile("v_lshrrev_b32 %0, 13, %0" : "+v"(x[i]))
        if (OP == 14) C8(X)
#undef X
#define X(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 15) C8(X)
#undef X
#define X(i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 16) C8(X)
#undef X
#define X(i) asm volatile("v_min_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]))
        if (OP == 17) C8(X)
#undef X
#define X(i) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "s"(c))
        if (OP == 18) C8(X)
#undef X
#define X(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 19) C8(X)
#undef X
#define X(i) asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[i]) : "s"(c))
        if (OP == 20) C8(X)
#undef X
#define X(i) asm volatile("v_mul_f32 %0, %0, %0" : "+v"(x[i]))
        if (OP == 21) C8(X)
#undef X
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, -1.0" : "+v"(x[i]) : "v"(v))
        if (OP == 22) C8(X)
#undef X
#define X(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y[i]) : "v"(x[i]), "v"(v) : "vcc")
        if (OP == 23) C8(X)
#undef X
#define X(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 24) C8(X)
#undef X
#define X(i) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 25) C8(X)
#undef X
#define X(i) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 26) C8(X)
#undef X
#define X(i) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 27) C8(X)
#undef X
#define X(i) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(y[i]))
        if (OP == 28) C8(X)
#undef X
#define X(i) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 29) C8(X)
#undef X
#define X(i) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(y[i]))
        if (OP == 30) C8(X)
#undef X
#define X(i) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(y[i]))
        if (OP == 31) C8(X)
#undef X
#define X(i) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(y[i]) : "v"(x[i]))
        if (OP == 32) C8(X)
#undef X
#define X(i) asm volatile("v_rcp_f32 %0, %0" : "+v"(x[i]))
        if (OP == 33) C8(X)
#undef X
#define X(i) asm volatile("v_sqrt_f32 %0, %0" : "+v"(x[i]))
        if (OP == 34) C8(X)
#undef X
#define X(i) asm volatile("v_cndmask_b32_e64 %0, %0, 0, %1" : "+v"(x[i]) : "s"(m))
        if (OP == 35) C8(X)
#undef X
#define X(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 36) C8(X)
#undef X
#define X(i) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 37) C8(X)
#undef X
#define X(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 38) C8(X)
#undef X
#define X(i) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x[i]))
        if (OP == 39) C8(X)
#undef X
#define X(i) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x[i]) : "v"(v))
        if (OP == 40) C8(X)
#undef X
#define X(i) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(x[i]))
        if (OP == 41) C8(X)
#undef X
#define X(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 42) C8(X)
#undef X
#define X(i) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 43) C8(X)
#undef X
#define X(i) asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 44) C8(X)
#undef X
#define X(i) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 45) C8(X)
#undef X
#define X(i) asm volatile("v_mov_b32 %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 46) C8(X)
#undef X
#define X(i) asm volatile("v_mov_b32 %0, 0x3f800001" : "+v"(x[i]))
        if (OP == 47) C8(X)
#undef X
#define X(i) asm volatile("v_not_b32 %0, %0" : "+v"(x[i]))
        if (OP == 48) C8(X)
#undef X
#define X(i) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 49) C8(X)
#undef X
#define X(i) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 50) C8(X)
#undef X
#define X(i) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(x[i]))
        if (OP == 51) C8(X)
#undef X
#define X(i) asm volatile("v_ldexp_f32 %0, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 52) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_class_f32 vcc, %0, %1" :: "v"(x[i]), "v"(v) : "vcc")
        if (OP == 53) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_lt_u32 vcc, %0, %1" :: "v"(x[i]), "v"(v) : "vcc")
        if (OP == 54) C8(X)
#undef X
#define X(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 55) C8(X)
#undef X
#define X(i) asm volatile("v_sub_f32 %0, %0, %1 clamp" : "+v"(x[i]) : "v"(v))
        if (OP == 56) C8(X)
#undef X
#define X(i) asm volatile("v_mul_f32 %0, -%0, |%1|" : "+v"(x[i]) : "v"(v))
        if (OP == 57) C8(X)
#undef X
#define X(i) asm volatile("v_add_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x[i]))
        if (OP == 58) C8(X)
#undef X
#define X(i) asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 59) C8(X)
#undef X
#define X(i) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 60) C8(X)
#undef X
#define X(i) asm volatile("v_lshl_or_b32 %0, %0, 2, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 61) C8(X)
#undef X
#define X(i) asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(y[i]))
        if (OP == 62) C8(X)
#undef X
#define X(i) asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(y[i]))
        if (OP == 63) C8(X)
#undef X
#define X(i) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]))
        if (OP == 64) C8(X)
#undef X
#define X(i) asm volatile("v_frexp_mant_f32 %0, %0" : "+v"(x[i]))
        if (OP == 65) C8(X)
#undef X
#define X(i) asm volatile("v_div_fixup_f32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(v))
        if (OP == 66) C8(X)
#undef X
#define X(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(v))
        if (OP == 67) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n\ts_nop 1\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(x[i]) : "v"(v) : "vcc")
        if (OP == 68) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_gt_f32_e64 %2, %0, %1\n\tv_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(x[i]) : "v"(v), "s"(m))
        if (OP == 69) C8(X)
#undef X
#define X(i) asm volatile("v_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"(x[i]) : "v"(v))
        if (OP == 70) C8(X)
#undef X
#define X(i) asm volatile("v_fma_f32 %0, %0, %1, 1.0\n\tv_fma_f32 %0, %0, %1, 1.0" : "+v"(x[i]) : "v"(v))
        if (OP == 71) C8(X)
#undef X
#define X(i) asm volatile("s_mov_b64 vcc, %2\n\tv_cndmask_b32_e32 %0, %1, %0, vcc" : "+v"(x[i]) : "v"(v), "s"(m) : "vcc")
        if (OP == 72) C8(X)
#undef X
#define X(i) asm volatile("s_mov_b64 s[40:41], %2\n\tv_cndmask_b32_e64 %0, %1, %0, s[40:41]" : "+v"(x[i]) : "v"(v), "s"(m) : "s40", "s41")
        if (OP == 73) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_gt_f32 vcc, %0, %1\n\ts_and_b64 vcc, vcc, exec\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(x[i]) : "v"(v) : "vcc")
        if (OP == 74) C8(X)
#undef X
#define X(i) asm volatile("v_cmp_gt_f32_e64 s[40:41], %0, %1\n\ts_and_b64 s[40:41], s[40:41], exec\n\tv_cndmask_b32_e64 %0, %1, %0, s[40:41]" : "+v"(x[i]) : "v"(v) : "s40", "s41")
        if (OP == 75) C8(X)
#undef X
    }
    uint32_t r = (uint32_t)m;
    for (int i = 0; i < 8; ++i) r ^= x[i] ^ (uint32_t)y[i] ^ (uint32_t)(y[i] >> 32);
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

constexpr int kOps = 76;
const char *kNames[kOps] = {
    "v_fma_f32 v,v,v",     "v_fma_f32 v,s,v",      "v_mul_f32 lit,v"  ,       "v_fma_f32 v,2.0,v",
    "v_cndmask vcc",       "v_cndmask_e64 s[]",    "v_cmp_lt_f32 vcc",        "v_cmp_lt_f32_e64 s[]",
    "v_add_u32 v,v",       "v_mul_lo_u32 v,v",     "v_mad_u64_u32 s[],v,v",   "v_alignbit_b32 v,v,v",
    "v_cvt_f32_u32",       "v_min_f32 lit,v",      "v_lshrrev_b32 13,v",      "v_xor_b32 v,v",
    "v_add3_u32",          "v_min_u32_dpp quad",   "v_mov_b32 v,s",           "v_add_f32 v,v",
    "v_add_f32 s,v",       "v_mul_f32 v,v",        "v_fma_f32 v,v,-1.0",      "v_mad_u64_u32 vcc,v,v",
    "v_mul_hi_u32 v,v",    "v_max_f32 v,v",        "v_sub_f32 v,v",           "v_med3_f32",
    "v_lshlrev_b64",       "v_lshl_add_u32",       "v_fma_f64",               "v_mul_f64",
    "v_cvt_f64_f32",       "v_rcp_f32",            "v_sqrt_f32",              "v_cndmask_e64 0,s[]",
    "v_and_b32 v,v", "v_or_b32 v,v", "v_sub_u32 v,v", "v_lshlrev_b32 3,v", "v_lshrrev_b32 v,v", "v_bfe_u32", "v_mul_u32_u24 v,v", "v_min_u32 v,v", "v_max_i32 v,v", "v_fmac_f32 v,v", "v_mov_b32 v,v", "v_mov_b32 v,lit", "v_not_b32", "v_bfi_b32", "v_perm_b32", "v_cvt_f32_i32", "v_ldexp_f32 v,v", "v_cmp_class_f32", "v_cmp_lt_u32 vcc", "v_add_co_u32 vcc", "v_sub_f32 clamp", "v_mul_f32 neg/abs", "v_add_f32_dpp", "v_max3_f32", "v_or3_b32", "v_lshl_or_b32", "v_pk_mul_f32", "v_pk_add_f32", "v_exp_f32", "v_frexp_mant_f32", "v_div_fixup_f32", "v_cndmask vcc (no clobber)",
    "cmp vcc + cndmask vcc (pair)", "cmp s[] + cndmask s[] (pair)", "cndmask_e32 vcc, no clobber", "fma pair (reference)",
    "s_mov vcc + cndmask_e32 vcc", "s_mov s[] + cndmask_e64 s[]", "cmp vcc + s_and vcc + cndmask vcc", "cmp s[] + s_and s[] + cndmask_e64"};

template <int OP>
static float run(uint32_t *out, int blocks)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    probe<OP><<<blocks, 256>>>(out, 0x3f800001u);
    (void)hipEventRecord(a);
    probe<OP><<<blocks, 256>>>(out, 0x3f800001u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms;
}

template <int... I>
static void run_all(uint32_t *out, int blocks, float *ms, int first, double insts, int clk,
                    std::integer_sequence<int, I...>)
{
    // one line per op as it completes (a slow shape shows up before the rest)
    ((I >= first ? (ms[I] = run<I>(out, blocks),
                    printf("%-32s %.3f ms  %.2f cycles/wave-inst/SIMD at %.0f MHz\n", kNames[I], ms[I],
                           ms[I] * 1e-3 * clk * 1e3 / insts, clk / 1e3),
                    fflush(stdout), 0)
                 : 0),
     ...);
}

int main(int argc, char **argv)
{
    int clk = 0, cus = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    uint32_t *out;
    (void)hipMalloc(&out, sizeof(uint32_t) * 256 * blocks);
    float ms[kOps];
    const double insts = 8.0 * kIters * 8;  // per SIMD: waves x iterations x chains
    run_all(out, blocks, ms, argc > 1 ? atoi(argv[1]) : 0, insts, clk, std::make_integer_sequence<int, kOps>{});
    (void)hipFree(out);
    return 0;
}
