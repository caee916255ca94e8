// rt_kernel.hip — the hot path: per-pixel path tracing (color -> closest hit -> scatter) as a
// persistent HIP megakernel for gfx950 (CDNA4), plus the ordered sample-accumulation pass.
//
// Semantics are the reference CPU path, bit for bit in the exact variants:
//   app::color                      src/main.cxx:52-75
//   app::background_color / mix     src/main.cxx:47-50, src/math.hxx:325-329
//   raytracer::hit_world/intersect  src/raytracer.hxx:52-118
//   raytracer::apply_material       src/raytracer.hxx:120-199
//   raytracer::random_in_unit_sphere, schlick  src/raytracer.hxx:32-50
//   raytracer::camera::ray          src/camera.hxx:46-57
//   pixel/sample driver + reduce    src/main.cxx:185-207
// Every binary32 op is separately rounded in the reference's order: this file is compiled
// with -ffp-contract=off and without fast-math, so div/sqrt are the correctly rounded
// sequences and NaN semantics (total internal reflection, src/math.hxx:308) survive.
//
// Execution model: one lane owns one work item (a block of 4 samples or
// one tail sample of one pixel) at a time. Every loop iteration traces ONE segment for every
// lane whose path is alive; lanes whose path ended refill from a per-wave item cursor
// (ballot + mbcnt prefix, no atomics), and the wave refills its cursor from one of 8 chunk
// queues. So lanes never idle waiting for the longest path of their wave (active-lane
// compaction across bounces) and the sphere loop always runs with the wave's live lanes.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

#include "rt_device.h"

namespace rt {

#define RT_TMIN 0.008f   // raytracer.hxx:98 kMIN
#define RT_TMAX FLT_MAX  // raytracer.hxx:97 kMAX

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return {x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ f3 adds(f3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float length(f3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ f3 normalize(f3 a)                    // math.hxx:219-227
{
    float l = length(a);
    return fabsf(l) > FLT_MIN ? a / l : a;
}
__device__ __forceinline__ f3 reflect(f3 I, f3 N) { return I - (N * dot(N, I)) * 2.f; } // math.hxx:294-298
__device__ __forceinline__ float sqrt_scaled(float x);
__device__ __forceinline__ f3 refract(f3 I, f3 N, float eta)                          // math.hxx:300-309
{
    const float d = dot(N, I);
    const float k = 1.f - eta * eta * (1.f - d * d);
    return (I * eta - adds(N * sqrt_scaled(k), d * eta)) * (k >= 0.f ? 1.f : 0.f);  // k <= 1
}

// Diagnostic counters (STATS builds only; see rt_scene_debug_counters): per-lane tallies
// plus wave-level ones counted by the first active lane.
struct Dbg {
    uint32_t wave_blocks, lane_blocks, wave_roots, lane_roots, wave_member_blocks;
    uint32_t ev[kDbgEvents];  // executions of the code blocks below by the wave (rt_scene_debug_events)
};
__device__ __forceinline__ bool first_active_lane()
{
    return (threadIdx.x & 63u) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63u);
}
// block-execution events (STATS builds): counted once per wave each time the block runs
enum DbgEvent : uint32_t {
    EV_ITER, EV_REFILL_TRIP, EV_FRESH, EV_REJECT_TRIP, EV_LENS_DONE, EV_SCATTER_DONE, EV_ROOT_GATE_PASS,
    EV_SUPER, EV_SUPER_PASS, EV_CLUSTER_REQ, EV_TRANSPOSED, EV_T_ROUND, EV_T_FAR, EV_PER_LANE_MEMBERS,
    EV_SKY, EV_HIT, EV_LAMBERT, EV_UNIT_DIR, EV_DIELECTRIC, EV_STORE, EV_METAL_ABSORB,
    EV_LIVE_LANES,  // live lanes summed over wave iterations
    EV_DRY_ITER,    // wave iterations after the item queues ran dry (the drain)
    EV_DRY_LANES,   // live lanes summed over those
    EV_ISO_LANES,   // lanes that skipped the cluster walk (isolated hint sphere), summed over iterations
    EV_WALK_SKIPPED,  // wave iterations with segments whose cluster walk no lane needed
    EV_WALK1, EV_WALK2, EV_WALK4, EV_WALK8,  // wave iterations whose walk 1, 2, 3-4, 5-8 lanes need
    EV_PAIR_SUM,   // (lanes) pair sums stored by the main launch (both samples ended there)
    EV_BOTH_MEET,  // (lanes) pair sums formed in the deep launch by the second of two queued samples
    EV_COUNT
};
static_assert(EV_COUNT <= kDbgEvents, "event counters");
#define RT_EV(e)                                          \
    do {                                                  \
        if (STATS && first_active_lane()) ++dbg.ev[(e)]; \
    } while (0)

// The lane mask of a predicate. Votes are taken on single compares only: the compiler turns the
// vote of a compare into one scalar AND with exec, but materialises any other predicate (an AND
// of compares, a value carried across blocks) as 0/1 in a VGPR and compares it again, two extra
// half-rate VALU operations; compound conditions are formed from masks instead.
__device__ __forceinline__ uint64_t ballot(bool x) { return __builtin_amdgcn_ballot_w64(x); }
__device__ __forceinline__ uint32_t lanes(bool x) { return (uint32_t)__popcll(ballot(x)); }

// Bounds check of the instrumented kernel (STATS; rt_device.h kDbgError): an index at or past its
// bound is recorded (the first one wins) and replaced by 0, so the diagnostic never makes the
// access it reports. The product kernels compile this to the index itself.
template <bool STATS>
__device__ __forceinline__ uint32_t checked(uint32_t i, uint32_t bound, uint32_t code, unsigned long long *dbg)
{
    if (STATS && i >= bound) {
        atomicCAS(dbg + kDbgError, 0ull, ((unsigned long long)code << 32) | i);
        return 0u;
    }
    return i;
}

// ---- RNG: PCG32 XSH-RR per (pixel, sample) stream; the increment is wave-uniform ---------
constexpr uint64_t kPcgMul = 6364136223846793005ULL;
__device__ __forceinline__ uint32_t pcg_out(uint64_t old)
{
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
}
__device__ __forceinline__ uint32_t pcg_next(uint64_t &state, uint64_t inc)
{
    uint64_t old = state;
    state = old * kPcgMul + inc;
    return pcg_out(old);
}
__device__ __forceinline__ uint64_t pcg_seed(uint64_t initstate, uint64_t inc)
{
    uint64_t st = inc;  // state = 0; next() -> 0 * M + inc
    st += initstate;
    return st * kPcgMul + inc;
}
// libstdc++ generate_canonical<float,24> over a 32-bit engine: float(x) / 2^32, kept < 1.
// float(x) rounds up to 2^32 for the top 128 words; clamping it to the largest float below,
// 2^32 - 256, before the exact scaling gives the same 0x1.fffffep-1.
__device__ __forceinline__ float canonical(uint64_t &st, uint64_t inc)
{
    return fminf((float)pcg_next(st, inc), 0x1.fffffep31f) * 0x1p-32f;
}
// canonical() * 2.f + -1.f (raytracer.hxx:35-37): the product is exact, so the result is the
// one rounding of clamp(float(x)) * 2^-31 - 1, i.e. a single FMA.
__device__ __forceinline__ float canonical_pm1(uint64_t &st, uint64_t inc)
{
    return fmaf(fminf((float)pcg_next(st, inc), 0x1.fffffep31f), 0x1p-31f, -1.f);
}
// RN(a / b) for a per-render divisor b (the image width or height): one reciprocal rb = RN(1/b)
// and one FMA correction (Markstein) when the host has checked, for this b, that the sequence
// reproduces the IEEE quotient for every float mantissa (rt_host.cpp exact_by_reciprocal: the
// result then holds for every normal a >= 0, the scaling by powers of two being exact);
// otherwise the IEEE division.
__device__ __forceinline__ float div_const(float a, float b, float rb, bool fast)
{
    if (fast) {
        const float q0 = a * rb;
        const float r = fmaf(-q0, b, a);
        return fmaf(r, rb, q0);
    }
    return a / b;
}
// raytracer.hxx:32-43. `length(p) > 1` is evaluated as `norm(p) > 1 + 2^-23`: with a
// correctly rounded sqrt the two agree for every non-negative float (checked exhaustively,
// tests/test_numerics_cpu.py), and the loop runs as long as its slowest lane.
__device__ __forceinline__ f3 random_in_unit_sphere(uint64_t &st, uint64_t inc)
{
    f3 p;
    do {
        float x = canonical_pm1(st, inc);
        float y = canonical_pm1(st, inc);
        float z = canonical_pm1(st, inc);
        p = mk(x, y, z);
    } while (p.x * p.x + p.y * p.y + p.z * p.z > 0x1.000002p+0f);
    return p;
}

// At most RT_REJECT_CAP attempts of raytracer.hxx:32-43 in this call: `got` tells whether one
// was accepted; if not, st is left after the failed attempts' draws and the caller resumes the
// same sequence next time. The wave runs this as long as its unluckiest lane, up to the cap.
#ifndef RT_REJECT_CAP
#define RT_REJECT_CAP 4  // 0: unbounded (the loop runs until every lane accepts)
#endif
template <bool STATS, int CAP = RT_REJECT_CAP>
__device__ __forceinline__ f3 random_in_unit_sphere_capped(uint64_t &st, uint64_t inc, bool &got, Dbg &dbg)
{
    if (CAP == 0) {
        got = true;
        return random_in_unit_sphere(st, inc);
    }
    // p is written on every attempt a lane makes: a lane that accepted has left the loop, so
    // later attempts do not touch its p, and no per-attempt select is needed (p of a lane that
    // did not accept is not used)
    // The LCG multiplier's halves and the 2^-31 scale sit in VGPRs for the loop (three moves
    // of literals): on gfx950 a VALU operation reading an SGPR issues at half rate
    // (scripts/ubench_int.hip), and the compiler would keep these uniform constants in SGPRs.
    uint32_t m_lo = (uint32_t)kPcgMul, m_hi = (uint32_t)(kPcgMul >> 32);
    float k31 = 0x1p-31f;
    asm volatile("" : "+v"(m_lo), "+v"(m_hi), "+v"(k31));
    const uint64_t mul = ((uint64_t)m_hi << 32) | m_lo;
    auto draw = [&]() {
        const uint64_t old = st;
        st = old * mul + inc;
        return fmaf(fminf((float)pcg_out(old), 0x1.fffffep31f), k31, -1.f);  // canonical_pm1
    };
    f3 p;
    got = false;
#pragma unroll
    for (int k = 0; k < (CAP > 0 ? CAP : 1); ++k) {
        RT_EV(EV_REJECT_TRIP);
        p.x = draw();
        p.y = draw();
        p.z = draw();
        if (!(p.x * p.x + p.y * p.y + p.z * p.z > 0x1.000002p+0f)) {
            got = true;
            break;
        }
    }
    return p;
}

// raytracer.hxx:45-50. std::pow(float,int) promotes to double: r0 = x^2 is exact in double;
// (1-cos)^5 is formed as y^4 * y with y^4 = y^2*y^2 split exactly by an FMA, so the double
// product is within a few 1e-17 relative of glibc's pow before the final cast to float.
// xf = (1 - ri) / (1 + ri) in binary32 (per sphere and side, from the host).
__device__ __forceinline__ float schlick_x(float xf, float c)
{
    double x = (double)xf;
    double r0 = x * x;
    double y = (double)(1.f - c);
    double y2 = y * y;                  // exact (24-bit * 24-bit)
    double y4 = y2 * y2;
    double y4lo = fma(y2, y2, -y4);     // exact residual
    double y5 = fma(y4, y, y4lo * y);
    return (float)(r0 + (1.0 - r0) * y5);
}
__device__ __forceinline__ float schlick(float ri, float c) { return schlick_x((1.f - ri) / (1.f + ri), c); }

// ---- work decomposition ----------------------------------------------------------------
template <class UD>
__device__ __forceinline__ uint32_t udiv(uint32_t n, const UD &u)
{
    const uint32_t t = __umulhi(n, u.m);
    return (t + ((n - t) >> u.s1)) >> u.s2;
}

// pixel (x, packed row rr) of enumeration position i; perm: the pass's block permutation
// (KParams::block_perm) or null
#ifndef RT_PERM_SCALAR
#define RT_PERM_SCALAR 1  // A/B build switch: the block permutation read through the scalar cache
#endif
template <class FC>
__device__ __forceinline__ void pixel_of(const FC &fc, uint32_t i, uint32_t &x, uint32_t &rr, const uint32_t *perm)
{
    if (perm) {
        // the active lanes' positions lie in one or two blocks nearly always (fresh lanes take
        // consecutive items of one tile at one sample): the first lane's block through a scalar
        // load, vector loads only for lanes in another block
        const uint32_t b = i >> 6;
        uint32_t nb;
        if (RT_PERM_SCALAR) {
            const uint32_t b0 = __builtin_amdgcn_readfirstlane(b);
            nb = perm[b0];
            if (b != b0) nb = perm[b];
        } else {
            nb = perm[b];
        }
        i = (nb << 6) | (i & 63u);
    }
    const uint32_t W = fc.W, tiled_rows = fc.tiled_rows, tiles_x = fc.tiles_x;
    const uint32_t tiled_px = tiled_rows * W;
    if (i < tiled_px) {
        uint32_t t = i >> 6, w = i & 63u;
        uint32_t ty = udiv(t, fc.div_tiles_x), tx = t - ty * tiles_x;
        const uint32_t lw = fc.tile_lw;
        x = (tx << lw) + (w & ((1u << lw) - 1u));
        rr = (ty << (6u - lw)) + (w >> lw);
    } else {
        uint32_t j = i - tiled_px;
        rr = udiv(j, fc.div_W);
        x = j - rr * W;
        rr += tiled_rows;
    }
}

// ---- closest hit (raytracer.hxx:94-118) -------------------------------------------------
// The reference tests every sphere on (kMIN, kMAX) and keeps the first minimum in index
// order (stable_partition + min_element with a strict '<'). Here every sphere that is
// tested yields the reference's per-sphere candidate (near root if in range, else far root,
// raytracer.hxx:62-90) and candidates are compared on (t, original index) lexicographically
// — the same minimum whatever order spheres are visited in, so the scene may be reordered
// into spatial clusters. Spheres come 8 at a time: 8 discriminants, one
// max reduction (NaN never wins) and the root work only when some lane needs it.
struct Hit {  // the closest candidate so far as hit_key(t, original index); ~0 = none
    uint64_t key;
    __device__ float t() const { return __uint_as_float((uint32_t)(key >> 32)); }
    __device__ uint32_t id() const { return (uint32_t)key; }
};
constexpr uint64_t kNoHit = 0x7f7fffffffffffffull;  // t = kMAX, index = none
// kNoHit made in VGPRs where it is used: left to itself the allocator keeps the constant in a
// VGPR pair for the whole kernel, and at 7 waves per SIMD (72 VGPRs) spills it to scratch
__device__ __forceinline__ uint64_t no_hit()
{
    uint32_t lo = 0xffffffffu, hi = 0x7f7fffffu;
    asm volatile("" : "+v"(lo), "+v"(hi));
    return ((uint64_t)hi << 32) | lo;
}
// this lane's slot of a per-thread LDS array: the wave's first slot (a scalar) plus the lane
// id, recomputed at each use (keeping threadIdx.x * 16 live across the loop costs a VGPR,
// which at 7 waves per SIMD is spilled to scratch)
__device__ __forceinline__ uint32_t thread_slot(uint32_t wave_base)
{
    uint32_t l;  // the lane id, formed here (the builtins' result is hoisted and kept live)
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return wave_base + l;
}

// Work counters of one wave (wave-uniform, scalar registers): segments traced and the
// lane-level ray-sphere and cluster-box tests executed, summed from ballots in uniform control
// flow (a test the wave runs for k requesting lanes counts k).
// Only the counting instantiation (COUNT, used when the caller asks for the counters) keeps them.
template <bool COUNT>
struct WaveTally {
    uint64_t seg = 0, sph = 0, box = 0;
    __device__ __forceinline__ void add_seg(uint32_t n) { if (COUNT) seg += n; }
    __device__ __forceinline__ void add_sph(uint64_t n) { if (COUNT) sph += n; }
    __device__ __forceinline__ void add_box(uint32_t n) { if (COUNT) box += n; }
};
// t in (kMIN, kMAX), the reference's test (raytracer.hxx:63-64,76-77): positive binary32 values
// are ordered as their bit patterns, and as unsigned integers every negative value and every
// NaN lies outside the open interval of patterns, so one subtract and one compare decide it.
__device__ __forceinline__ bool in_range(float t)
{
    constexpr uint32_t lo = 0x3c03126fu;  // bits of RT_TMIN (0.008f)
    constexpr uint32_t hi = 0x7f7fffffu;  // bits of RT_TMAX (FLT_MAX)
    return __float_as_uint(t) - (lo + 1u) < hi - lo - 1u;
}
// A candidate as a 64-bit key, bits(t) << 32 | original index: for t > 0 (or NaN, which loses to
// every valid t) the unsigned key order is the (t, index) order of closest_hit.
__device__ __forceinline__ uint64_t hit_key(float t, uint32_t id)
{
    return ((uint64_t)__float_as_uint(t) << 32) | id;
}

// ---- the root of a candidate (raytracer.hxx:62-90) -----------------------------------------
// The IEEE forms of sqrtf and of division, as the compiler expands them, scale operands whose
// exponents are extreme and fix up special values; when neither can occur they reduce to shorter
// exact sequences. Per ray segment the divisor a = |d|^2 gets its refined reciprocal once (the
// divisor-only head of the division sequence). fd (wave-uniform) says the short forms give the
// IEEE bits for every lane: the scene lies within 2^19 of the origin (KParams::fast_roots: then
// |oc| <= 2^21 and every in-range root is below 2^43) and every active lane has a in
// [2^-40, 2^40], so no root division needs scaling (quotient exponents stay 96 below the
// numerator's) and every discriminant is below 2^96.
struct RayDiv {
    float a, y;  // divisor |d|^2 and its refined reciprocal
    uint32_t fd; // wave-uniform (a scalar, not a lane predicate): the short forms are exact for every lane
};
__device__ __forceinline__ RayDiv ray_div(float a, uint64_t active, uint32_t fast_roots)
{
    const float y0 = __builtin_amdgcn_rcpf(a);
    const float y = fmaf(fmaf(-a, y0, 1.f), y0, y0);
    const uint64_t ok = ballot(a >= 0x1p-40f) & ballot(a <= 0x1p40f);  // NaN: neither
    return {a, y, (uint32_t)__builtin_amdgcn_readfirstlane((fast_roots != 0u && !(active & ~ok)) ? 1u : 0u)};
}
// n / a: the IEEE sequence (v_div_scale, rcp + refinement, two FMA corrections, v_div_fmas,
// v_div_fixup) with no scaling and no special value, i.e. its two corrections
__device__ __forceinline__ float div_ray(float n, const RayDiv &r)
{
    const float q0 = n * r.y;
    const float q1 = fmaf(fmaf(-r.a, q0, n), r.y, q0);
    return fmaf(fmaf(-r.a, q1, n), r.y, q1);
}
// correctly rounded sqrt for 0 < x < 2^96: the compiler's IEEE expansion (v_sqrt_f32, then the
// one-ulp neighbours checked by FMA residuals) always run on x * 2^32 and scaled back by 2^-16,
// both exact, so the result is that of the expansion's own small-input path for every such x
__device__ __forceinline__ float sqrt_scaled(float x)
{
    const float xs = x * 0x1p32f;
    const float s = __builtin_amdgcn_sqrtf(xs);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
    const float sup = __uint_as_float(__float_as_uint(s) + 1u);
    float r = fmaf(-sdn, s, xs) <= 0.f ? sdn : s;
    r = fmaf(-sup, s, xs) > 0.f ? sup : r;
    return r * 0x1p-16f;
}
// r.fd, re-read as a scalar at each use: left to itself the compiler hoists `fd != 0` out of the
// sphere loops as a lane predicate and rebuilds its negation per use with two VALU operations
__device__ __forceinline__ bool fast_div(const RayDiv &r)
{
    uint32_t f = r.fd;  // uniform by construction (ray_div): an SGPR, no readfirstlane here
    asm volatile("" : "+s"(f));
    return f != 0u;
}
// n / r for the three components of n by the short form, with r's refined reciprocal formed once.
// The caller has checked that no operand takes the IEEE sequence's scaling or fix-up paths:
// r in [2^-40, 2^20], every |n_i| in [2^-100, 2^21] (so no zero, whose sign the short form can
// lose, and no quotient below 2^-126).
__device__ __forceinline__ f3 div3_short(f3 n, float r)
{
    const float y0 = __builtin_amdgcn_rcpf(r);
    const RayDiv rr{r, fmaf(fmaf(-r, y0, 1.f), y0, y0), 1u};
    return mk(div_ray(n.x, rr), div_ray(n.y, rr), div_ray(n.z, rr));
}
// every active lane's |n_i| >= 2^-100 (a wave-uniform answer; one min3 and one compare per lane)
__device__ __forceinline__ bool all_lanes_min_abs_ok(f3 n)
{
    return !ballot(!(fminf(fminf(fabsf(n.x), fabsf(n.y)), fabsf(n.z)) >= 0x1p-100f));
}
// the near root (-b - sqrt(disc)) / a and its sqrt, raytracer.hxx:62-63; FD: 1 the short forms
// (the caller has branched on fast_div), 0 the IEEE forms, -1 a branch on fast_div here
template <int FD = -1>
__device__ __forceinline__ float near_root(float b, float disc, const RayDiv &r, float &q)
{
    if (FD == 1 || (FD < 0 && fast_div(r))) {
        q = sqrt_scaled(disc);
        return div_ray(-b - q, r);
    }
    q = sqrtf(disc);
    return (-b - q) / r.a;
}
// the far root (-b + sqrt(disc)) / a, raytracer.hxx:76
template <int FD = -1>
__device__ __forceinline__ float far_root(float b, float q, const RayDiv &r)
{
    return (FD == 1 || (FD < 0 && fast_div(r))) ? div_ray(-b + q, r) : (-b + q) / r.a;
}
template <int B> struct IntC { static constexpr int value = B; };

#ifndef RT_GROUND1
#define RT_GROUND1 1
#endif
#ifndef RT_ROOT_HOIST
#define RT_ROOT_HOIST 5  // bit 0: blocks of 8, bit 1: of 4, bit 2: single spheres (8 and 4 together spill)
#endif
template <bool FAST, bool STATS, int N = 8>
__device__ __forceinline__ void test_block8(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx, uint32_t i,
                                            f3 o, f3 d, const RayDiv &rd, Hit &h, Dbg &dbg)
{
    const float a = rd.a;
    float bq[N], dq[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const float4 s = geo[i + k];
        const float ocx = o.x - s.x, ocy = o.y - s.y, ocz = o.z - s.z;       // raytracer.hxx:55
        float b, c;
        if (FAST) {  // contracted: 11 VALU per sphere
            b = fmaf(ocx, d.x, fmaf(ocy, d.y, ocz * d.z));
            c = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -s.w)));
            dq[k] = fmaf(b, b, -(a * c));
        } else {     // the reference's rounding, op by op: 17 VALU per sphere
            b = ocx * d.x + ocy * d.y + ocz * d.z;                           // :57
            c = ocx * ocx + ocy * ocy + ocz * ocz - s.w;                     // :58
            dq[k] = b * b - a * c;                                           // :60
        }
        bq[k] = b;
        if (N == 1) {
            // The always-tested spheres (the ground): a ray leaving the sphere (b > 0) from
            // outside it (c >= 0) has no candidate unless rounding makes the far root reach
            // kMIN: with a c >= 0 the discriminant is at most RN(b^2), so its correctly rounded
            // root q is at most b + ulp(b), the near root is negative and the far root
            // RN((q - b) / a) <= RN(ulp(b) / a) < kMIN when b 2^-22 < kMIN a. Such lanes need
            // no root work: their discriminant is set to -1 (no candidate, as computed), and a
            // wave of them (upward rays from above the ground: the sky) skips it.
            if (b > 0.f && c >= 0.f && b * 0x1p-22f < RT_TMIN * a) dq[k] = -1.f;
        }
    }
    // pairwise max tree (NaN never wins)
    float mq[N];
#pragma unroll
    for (int k = 0; k < N; ++k) mq[k] = dq[k];
#pragma unroll
    for (int w = N / 2; w >= 1; w /= 2)
#pragma unroll
        for (int k = 0; k < w; ++k) mq[k] = fmaxf(mq[k], mq[k + w]);
    // Wave-uniform branches (ballots) around the root work, lane selects inside: a masked
    // lane costs the same issue slots as a computing one, and uniform branches need no
    // exec-mask save/restore. Lanes without a positive discriminant take the root of -1
    // (NaN), so their candidate is NaN, whose key never wins (NaN bits order above every
    // finite t): no predicate is carried to the key update, which is selected by the key
    // compare alone. (Formed as `pos && kt < h.key`, the mask would be ANDed into VCC by a
    // scalar op, and a VALU read of a VCC that a scalar op wrote stalls ~20 cycles on gfx950,
    // scripts/ubench_int.hip.)
    // The root form is chosen once for the block's roots (one uniform branch, not one per root)
    auto roots = [&](auto fdc) {
        constexpr int FD = decltype(fdc)::value;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const bool pos = dq[k] > 0.f;                                    // :62
            const uint64_t posm = ballot(pos);
            if (posm) {
                if (STATS) { dbg.lane_roots += pos; if (first_active_lane()) ++dbg.wave_roots; }
                const float dk = pos ? dq[k] : -1.f;
                float q;
                float t = near_root<FD>(bq[k], dk, rd, q);                   // :63
                const bool ok = in_range(t);
                if (posm & ~ballot(ok)) {
                    const float t2 = far_root<FD>(bq[k], q, rd);             // :76
                    t = ok ? t : (in_range(t2) ? t2 : __builtin_nanf(""));
                } else {
                    t = ok ? t : __builtin_nanf("");
                }
                const uint64_t kt = hit_key(t, sidx[i + k]);
                if (kt < h.key) h.key = kt;
            }
        }
    };
    if (ballot(mq[0] > 0.f)) {
        if (STATS) { ++dbg.lane_blocks; if (first_active_lane()) ++dbg.wave_blocks; }
        constexpr bool hoist = (RT_ROOT_HOIST >> (N == 8 ? 0 : N == 4 ? 1 : 2)) & 1;
        if (hoist && fast_div(rd)) roots(IntC<1>{});
        else roots(IntC<hoist ? 0 : -1>{});
    }
}

// Cluster culling: a lane tests a cluster's spheres only if its ray segment (kMIN, t_best]
// can reach the cluster's AABB grown by a pad that dominates every float error involved
// (1e-3 x (|o|_1 + max_c(|C|_1 + |e|_1)) against errors below 3e-4 of that),
// so a culled cluster never holds a sphere whose exact candidate could win: same bits.
#define RT_PAD_REL 1e-3f

// a list of spheres: blocks of 8, then 4, then single spheres (cluster member counts are
// multiples of 4; the always-tested list has its exact count, e.g. 1 for the ground)
template <bool FAST, bool STATS>
__device__ __forceinline__ void run_members(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx,
                                            uint32_t start, uint32_t cnt, f3 o, f3 d, const RayDiv &rd, Hit &h,
                                            Dbg &dbg)
{
    const uint32_t end = start + cnt;
    uint32_t i = start;
    for (; i + 8 <= end; i += 8) test_block8<FAST, STATS>(geo, sidx, i, o, d, rd, h, dbg);
    if (i + 4 <= end) { test_block8<FAST, STATS, 4>(geo, sidx, i, o, d, rd, h, dbg); i += 4; }
    for (; i < end; ++i) test_block8<FAST, STATS, 1>(geo, sidx, i, o, d, rd, h, dbg);
}

struct RayBox {  // per-segment constants of the padded slab test
    float ix, iy, iz, oix, oiy, oiz, aix, aiy, aiz, px, py, pz;
};
__device__ __forceinline__ bool box_pass(const RayBox &r, float4 c0, float4 c1, float t_lo, float t_hi)
{
    const float hx = fmaf(c0.w, r.aix, r.px), hy = fmaf(c1.x, r.aiy, r.py), hz = fmaf(c1.y, r.aiz, r.pz);
    const float tcx = fmaf(c0.x, r.ix, -r.oix), tcy = fmaf(c0.y, r.iy, -r.oiy), tcz = fmaf(c0.z, r.iz, -r.oiz);
    // tin <= tout && tout >= t_lo && tin <= t_hi, with t_lo < t_hi (no NaN arises: every
    // operand is finite or an infinity of one sign)
    const float tin = fmaxf(fmaxf(fmaxf(tcx - hx, tcy - hy), tcz - hz), t_lo);
    const float tout = fminf(fminf(fminf(tcx + hx, tcy + hy), tcz + hz), t_hi);
    return tin <= tout;
}

// Structure 7: the members of a passing cluster, tested transposed. A wave walks the union of
// its lanes' passing clusters, and in structure 5 every lane then runs the cluster's 16 tests
// while only the lanes whose segment reaches the cluster keep the results (20% of the lanes on
// config 3). Here, when at most kTransposeMax lanes request a cluster, all 64 lanes of the wave
// test (requesting ray, member) pairs instead — 4 rays x 16 members per round — and each
// ray's minimum over its 16 lanes comes back to its lane. Every pair yields the reference's
// per-sphere candidate (near root if in range, else far root, raytracer.hxx:62-90), and the
// candidates are combined by the (t, original index) minimum as key = bits(t) << 32 | index
// (t > 0, so the u64 order is that order): the same hit, in any order. Whole-wave code.
#ifndef RT_TRANSPOSE_LDS
#define RT_TRANSPOSE_LDS 16  // rays per transposed cluster the per-wave LDS holds
#endif
constexpr uint32_t kTransposeMax = RT_TRANSPOSE_LDS;  // KParams::transpose_max is clamped to this
// unsigned minimum over each row of 16 lanes: xor 1, xor 2 (quad permutes), then the half-row
// mirror and the row mirror leave every lane of a row with the row's minimum
// (the DPP moves carry the identity of min as their old value, so the compiler folds each into
// its v_min_u32 as a DPP operand)
__device__ __forceinline__ uint32_t min16_u32(uint32_t v)
{
#define RT_DPP_MIN(ctrl) v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, ctrl, 0xf, 0xf, false))
    RT_DPP_MIN(0xB1);
    RT_DPP_MIN(0x4E);
    RT_DPP_MIN(0x141);
    RT_DPP_MIN(0x140);
#undef RT_DPP_MIN
    return v;
}
// minimum key over each row of 16 lanes, in two 32-bit passes: the smallest t (as bits), then the
// smallest index among the lanes holding that t
__device__ __forceinline__ uint64_t min16_key(uint64_t k)
{
    const uint32_t tb = (uint32_t)(k >> 32);
    const uint32_t tm = min16_u32(tb);
    const uint32_t im = min16_u32(tb == tm ? (uint32_t)k : 0xffffffffu);
    return ((uint64_t)tm << 32) | im;
}
// per-wave LDS of the transposed tests: the requesting rays by rank; a ray's minimum key comes
// back in the last two words of its first record once its round is done (the round's rows read
// their rays before any row writes a key, and later rounds read other rays)
#ifndef RT_TKEY_SEPARATE
#define RT_TKEY_SEPARATE 0  // A/B build switch: the rows' keys in an array of their own (512 B more per workgroup)
#endif
struct TransposeLds {
    float4 ray[kTransposeMax][2];   // {o.x, o.y, o.z | key lo, a | key hi}, {d.x, d.y, d.z, refined 1/a}
#if RT_TKEY_SEPARATE
    uint64_t key[kTransposeMax];
#endif
};
template <bool FAST, bool STATS>
__device__ __forceinline__ void members_transposed(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx,
                                                   uint32_t start, uint32_t cnt, uint64_t M, bool req,
                                                   TransposeLds *tw, f3 o, f3 d, const RayDiv &rd, Hit &h,
                                                   Dbg &dbg)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m = (uint32_t)__popcll(M);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    if (req) {
        tw->ray[rank][0] = make_float4(o.x, o.y, o.z, rd.a);
        tw->ray[rank][1] = make_float4(d.x, d.y, d.z, rd.y);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t k = lane & 15u;          // member slot (slots >= cnt read beyond: masked)
    const float kth = k < cnt ? 0.f : __builtin_inff();  // slots past the cluster never test positive
    const float4 s = geo[start + k];
    const uint32_t sid = sidx[start + k];
    for (uint32_t r0 = 0; r0 < m; r0 += 4u) {
        RT_EV(EV_T_ROUND);
        const uint32_t r = r0 + (lane >> 4);
        const uint32_t rr = min(r, m - 1u);  // rows r >= m repeat ray m - 1; their keys are not stored
        const float4 q0 = tw->ray[rr][0], q1 = tw->ray[rr][1];
        const float ra = q0.w;                                              // |d|^2, as closest_hit
        const RayDiv rdr{ra, q1.w, rd.fd};
        const float ocx = q0.x - s.x, ocy = q0.y - s.y, ocz = q0.z - s.z;  // raytracer.hxx:55
        float b, disc;
        if (FAST) {
            b = fmaf(ocx, q1.x, fmaf(ocy, q1.y, ocz * q1.z));
            const float c = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -s.w)));
            disc = fmaf(b, b, -(ra * c));
        } else {
            b = ocx * q1.x + ocy * q1.y + ocz * q1.z;                     // :57
            const float c = ocx * ocx + ocy * ocy + ocz * ocz - s.w;     // :58
            disc = b * b - ra * c;                                         // :60
        }
        const bool pos = disc > kth;                                       // :62
        const uint64_t posm = ballot(pos);
        uint64_t key = ~0ull;
        if (posm) {
            const float dk = pos ? disc : -1.f;  // NaN candidate without a positive discriminant
            float q;
            float t = near_root(b, dk, rdr, q);                            // :63
            const bool ok = in_range(t);
            if (posm & ~ballot(ok)) {
                RT_EV(EV_T_FAR);
                const float t2 = far_root(b, q, rdr);                      // :76
                t = ok ? t : (in_range(t2) ? t2 : __builtin_nanf(""));
            } else {
                t = ok ? t : __builtin_nanf("");
            }
            // NaN keys (no candidate) lose to every valid key in the row minimum and in the
            // owner's update, like ~0 (test_block8)
            key = hit_key(t, sid);
        }
        key = min16_key(key);
        if (k == 0u && r < m) {
#if RT_TKEY_SEPARATE
            tw->key[r] = key;
#else
            tw->ray[r][0].z = __uint_as_float((uint32_t)key);
            tw->ray[r][0].w = __uint_as_float((uint32_t)(key >> 32));
#endif
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (req) {
#if RT_TKEY_SEPARATE
        const uint64_t kk = tw->key[rank];
#else
        const float4 q = tw->ray[rank][0];
        const uint64_t kk = ((uint64_t)__float_as_uint(q.w) << 32) | __float_as_uint(q.z);
#endif
        if (kk < h.key) h.key = kk;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <bool FAST, bool STATS, bool COUNT>
__device__ __forceinline__ void cluster_members7(bool req, uint64_t M, uint32_t scu_lane, const float4 *__restrict__ geo,
                                                 const uint32_t *__restrict__ sidx, TransposeLds *tw, uint32_t tmax,
                                                 f3 o, f3 d, const RayDiv &rd, Hit &h, Dbg &dbg, WaveTally<COUNT> &wt)
{
    // req: this lane's segment reaches the cluster box; M: the wave's mask of such lanes
    if (!M) return;
    RT_EV(EV_CLUSTER_REQ);
    const uint32_t scu = __builtin_amdgcn_readfirstlane(scu_lane);
    const uint32_t start = scu & 0xffffu, cnt = scu >> 16;
    wt.add_sph((uint64_t)__popcll(M) * cnt);
    if ((uint32_t)__popcll(M) <= min(tmax, kTransposeMax) && cnt <= 16u) {
        RT_EV(EV_TRANSPOSED);
        members_transposed<FAST, STATS>(geo, sidx, start, cnt, M, req, tw, o, d, rd, h, dbg);
    } else if (req) {
        RT_EV(EV_PER_LANE_MEMBERS);
        if (STATS && first_active_lane()) dbg.wave_member_blocks += (cnt + 7) / 8;
        run_members<FAST, STATS>(geo, sidx, start, cnt, o, d, rd, h, dbg);
    }
}

// One sphere's candidate for this lane's segment (raytracer.hxx:55-90, the op sequence of
// test_block8 on its geo entry {C, fl(r r)}) as a key, no_hit() without one. want: this lane
// asks (the others compute along and get no_hit()); t: the candidate's t when the key is valid.
template <bool FAST>
__device__ __forceinline__ uint64_t sphere_key(bool want, float4 s, uint32_t id, f3 o, f3 d, const RayDiv &rd, float &t)
{
    const float a = rd.a;
    const float ocx = o.x - s.x, ocy = o.y - s.y, ocz = o.z - s.z;            // raytracer.hxx:55
    float b, disc;
    if (FAST) {
        b = fmaf(ocx, d.x, fmaf(ocy, d.y, ocz * d.z));
        const float c = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -s.w)));
        disc = fmaf(b, b, -(a * c));
    } else {
        b = ocx * d.x + ocy * d.y + ocz * d.z;                               // :57
        const float c = ocx * ocx + ocy * ocy + ocz * ocz - s.w;             // :58
        disc = b * b - a * c;                                                // :60
    }
    const bool pos = want && disc > 0.f;                                     // :62
    const uint64_t posm = ballot(pos);
    t = 0.f;
    if (!posm) return no_hit();
    const float dk = pos ? disc : -1.f;  // NaN candidate without a positive discriminant
    float q;
    t = near_root(b, dk, rd, q);                                             // :63
    const bool ok = in_range(t);
    if (posm & ~ballot(ok)) {
        const float t2 = far_root(b, q, rd);                                 // :76
        t = ok ? t : (in_range(t2) ? t2 : __builtin_nanf(""));
    } else {
        t = ok ? t : __builtin_nanf("");
    }
    const uint64_t kt = hit_key(t, id);
    const uint64_t none = no_hit();
    return kt < none ? kt : none;  // a NaN key (no candidate) orders above kNoHit: none then
}

// The sphere a path last refracted into or reflected off inside (a dielectric hit), tested
// first: a ray trapped in a small glass sphere (the reference's refract, raytracer.hxx:158-194,
// keeps 0.17% of the samples bouncing up to max_depth, nearly all inside small dielectric
// spheres) then starts the walk with t_best at that sphere's far wall, and the padded boxes of
// every cluster its short segment does not reach are culled. The candidate is the reference's,
// so the (t, index) minimum is unchanged when the walk meets the sphere again. hint: this lane's
// last hit was a dielectric sphere, whose geo entry, original index (hid; kShortcut: the sphere
// has a shortcut word) and shortcut word (nbw) wait in the lane's LDS slots.
//
// The shortcut (rt_host.cpp shortcut_words; KParams::iso): when the segment (0, 1.002 t] up to
// the sphere's own candidate t lies in the ball |p - C|^2 <= fl(r r) kIsoR2Grow (both ends
// checked; the ball is convex), the host has shown that it misses the padded box of every
// clustered sphere but the sphere's at most two neighbours (none: "isolated"), whose slots nbw
// holds: the lane tests them here and needs no walk (`skip`; the always-tested spheres are still
// tested). A ray trapped in a small glass ball takes this path for every bounce.
//
// The neighbour slots of a lane that does not test a neighbour are 0, not its word's: a lane's
// word may be stale (left by an earlier path) or, before the lane's first dielectric hit, whatever
// the LDS held — bounded by that lane's own `skip` since fd383c3. The instrumented kernel (STATS)
// checks the slot against n_geo, starts every lane's word at 0x3fffffff (slots past any blob, no list), and
// with `unbounded` (KParams::diag_unbounded_nb) forms it the old way, so the check fires
// (tests/test_gpu_parity.py test_neighbour_slots_are_bounded).
template <bool FAST, bool STATS>
__device__ __forceinline__ uint64_t hint_candidate(bool hint, float4 s, uint32_t hid, uint32_t nbw,
                                                   const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx,
                                                   f3 o, f3 d, const RayDiv &rd, uint32_t iso, bool &skip,
                                                   uint32_t n_geo, uint32_t unbounded, unsigned long long *dbg)
{
    skip = false;
    float t;
    uint64_t key = sphere_key<FAST>(hint, s, hid & 0x7fffffffu, o, d, rd, t);
    if (iso && ballot(key < no_hit() && (int32_t)hid < 0)) {
        // a valid key implies hint; t then is finite and in range
        const float ocx = o.x - s.x, ocy = o.y - s.y, ocz = o.z - s.z;
        const float tq = t * 1.002f;  // the walk's bound, h.t() * 1.002f
        const float qx = fmaf(tq, d.x, ocx), qy = fmaf(tq, d.y, ocy), qz = fmaf(tq, d.z, ocz);
        const float r2k = s.w * kIsoR2Grow;
        const float o2 = ocx * ocx + ocy * ocy + ocz * ocz;
        const float q2 = qx * qx + qy * qy + qz * qz;
        skip = (int32_t)hid < 0 && key < no_hit() && o2 <= r2k && q2 <= r2k;
        // the neighbours (geo slots + 1 in nbw), tested by the lanes that skip the walk
        const uint32_t n0 = nbw & 0x7fffu, n1 = (nbw >> 15) & 0x7fffu;
        // (lanes that do not test a neighbour read slot 0: their word may be stale)
        if (ballot(skip && n0 != 0u)) {
            uint32_t g = (STATS && unbounded) ? (n0 ? n0 - 1u : 0u) : (skip && n0 ? n0 - 1u : 0u);
            g = checked<STATS>(g, n_geo, BC_HINT_NB, dbg);
            const uint64_t k = sphere_key<FAST>(skip && n0 != 0u, geo[g], sidx[g], o, d, rd, t);
            if (k < key) key = k;
        }
        if (ballot(skip && n1 != 0u)) {
            uint32_t g = (STATS && unbounded) ? (n1 ? n1 - 1u : 0u) : (skip && n1 ? n1 - 1u : 0u);
            g = checked<STATS>(g, n_geo, BC_HINT_NB, dbg);
            const uint64_t k = sphere_key<FAST>(skip && n1 != 0u, geo[g], sidx[g], o, d, rd, t);
            if (k < key) key = k;
        }
    }
    return key;
}

template <bool FAST, int CULL, bool STATS, bool COUNT, class KP>
__device__ __forceinline__ Hit closest_hit(const KP &p, const float4 *__restrict__ geo,
                                           const uint32_t *__restrict__ sidx, const float4 *__restrict__ clus, f3 o,
                                           f3 d, const RayDiv &rd, Dbg &dbg, WaveTally<COUNT> &wt, bool active,
                                           uint64_t am, TransposeLds *tw, uint64_t key0)
{
    // active: this lane traces a segment; am: the wave's mask of such lanes; key0: a candidate
    // already found for this segment (hint_candidate) or no_hit()
    Hit h{key0};
    // one always-tested sphere (the ground of the reference's scenes): its block without the
    // list's loop control
    if (RT_GROUND1 && p.n_always == 1u) test_block8<FAST, STATS, 1>(geo, sidx, 0, o, d, rd, h, dbg);
    else run_members<FAST, STATS>(geo, sidx, 0, p.n_always, o, d, rd, h, dbg);
    if (CULL) {
        // 1/x with its magnitude clamped to 1e30 (one med3; |x| < 1e-30 behaves as 1e-30 of
        // the same sign, zeros included): products with coordinates stay finite
        auto safe_rcp = [](float x) { return __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(x), -1e30f, 1e30f); };
        const float ix = safe_rcp(d.x), iy = safe_rcp(d.y), iz = safe_rcp(d.z);
        const float oix = o.x * ix, oiy = o.y * iy, oiz = o.z * iz;
        const float aix = fabsf(ix), aiy = fabsf(iy), aiz = fabsf(iz);
        const float pad = fmaf(RT_PAD_REL, fabsf(o.x) + fabsf(o.y) + fabsf(o.z), p.clus_pad);
        const float px = pad * aix, py = pad * aiy, pz = pad * aiz;
        const float t_lo = 0.5f * RT_TMIN;
        // Two levels under a root box, with whole-wave control (lanes predicated by `active`) so
        // that every lane can take part in a cluster's transposed member tests: the level-3 box
        // over every cluster gates the walk (a ray that misses the padded union box misses every
        // padded box inside it), a level-2 box covers kSuperClusters (8) consecutive clusters, and a passing
        // level-2 box's cluster boxes are tested in pairs against the current t_best.
        const RayBox rb{ix, iy, iz, oix, oiy, oiz, aix, aiy, aiz, px, py, pz};
        const float4 *sup = clus + (p.supers_offset - p.clus_offset);
        uint32_t n_supers = p.n_supers;
        if (!am) {
            n_supers = 0;  // every lane's segment is settled (isolated hint spheres)
        } else if (p.use_root) {
            wt.add_box(lanes(active));
            if (!(ballot(box_pass(rb, sup[2 * p.n_supers], sup[2 * p.n_supers + 1], t_lo, h.t() * 1.002f)) & am))
                n_supers = 0;
        }
        if (n_supers) RT_EV(EV_ROOT_GATE_PASS);
        for (uint32_t g = 0; g < n_supers; ++g) {
            RT_EV(EV_SUPER);
            const float4 s0 = sup[2 * g], s1 = sup[2 * g + 1];
            wt.add_box(lanes(active));
            const bool bs = box_pass(rb, s0, s1, t_lo, h.t() * 1.002f);
            const uint64_t spm = ballot(bs) & am;
            if (!spm) continue;
            const bool sp = bs & active;
            RT_EV(EV_SUPER_PASS);
            // its first cluster and the count the walk tests (up to its last non-empty one)
            const uint32_t sw = __builtin_amdgcn_readfirstlane(__float_as_uint(s1.w)), c0i = sw & 0xffffu, cn = sw >> 16;
            wt.add_box(cn * (uint32_t)__popcll(spm));
            for (uint32_t c = c0i; c < c0i + cn; c += 2) {
                const float tb_now = h.t() * 1.002f;
                const float4 a0 = clus[2 * c], a1 = clus[2 * c + 1], b0 = clus[2 * c + 2], b1 = clus[2 * c + 3];
                const bool ba = box_pass(rb, a0, a1, t_lo, tb_now), bb = box_pass(rb, b0, b1, t_lo, tb_now);
                const uint64_t pam = ballot(ba) & spm, pbm = ballot(bb) & spm;
                cluster_members7<FAST, STATS, COUNT>(ba & sp, pam, __float_as_uint(a1.w), geo, sidx, tw, p.transpose_max, o,
                                                     d, rd, h, dbg, wt);
                cluster_members7<FAST, STATS, COUNT>(bb & sp, pbm, __float_as_uint(b1.w), geo, sidx, tw, p.transpose_max, o,
                                                     d, rd, h, dbg, wt);
            }
        }
    }
    return h;
}

// ---- the megakernel ----------------------------------------------------------------------
// p[i] read from global memory, named as such (a float4 load from address space 1)
__device__ __forceinline__ float4 gld4(const float4 *p, uint32_t i)
{
    const __attribute__((address_space(1))) float *g = (const __attribute__((address_space(1))) float *)(p + i);
    return make_float4(g[0], g[1], g[2], g[3]);
}
// sphere ib's dielectric record {1 / ior, x(ior), x(1 / ior), shortcut word}, x(r) = (1 - r) / (1 + r),
// from LDS or global memory (the blob's tail)
template <int V, class KP>
__device__ __forceinline__ float4 dielectric_record(const KP &P, const float4 *blob, uint32_t ib)
{
    const uint32_t di = P.shade_offset + 2 * P.n_spheres + (P.n_spheres + 15u) / 16u + ib;
    if (V != V_EXACT_SCALAR && P.shade_lds) {
        const float4 r = blob[di];
        asm volatile("");  // no merged (flat) load with the global branch
        return r;
    }
    return gld4(P.blob, di);
}
#ifndef RT_MIN_WAVES_PER_SIMD
#define RT_MIN_WAVES_PER_SIMD 1  // measured: forcing 8 waves (64 VGPRs) spills and runs slower
#endif
// Structure 7 (the default) is held to 6 waves per SIMD: unhinted it takes 83 VGPRs (5 waves);
// hinted, the allocator keeps 79 and parks one 12-byte constant that only the metal-absorption
// path reloads (measured: 5.03-5.06 ms vs 5.19-5.24 per config-3 launch).
#ifndef RT_CULL7_WAVES
#define RT_CULL7_WAVES 7
#endif
template <int V, int CULL, bool STATS>
constexpr int kMinWaves = (CULL == 7 && !STATS) ? RT_CULL7_WAVES : RT_MIN_WAVES_PER_SIMD;
// the lone deep kernel's occupancy bound (waves per SIMD; 6: 3 workgroups of 8 waves per CU)
#ifndef RT_DEEP_REGHINT
#define RT_DEEP_REGHINT 0
#endif
#ifndef RT_DEEP_HOIST
// the lone deep kernel keeps its parameters in registers (106 SGPRs, no spills at its 6-wave bound;
// lone deep launch 0.341-0.351 vs 0.351-0.360 ms re-reading them, profiles/r05/deep/lone_deep_tmax.txt)
#define RT_DEEP_HOIST 1
#endif
#ifndef RT_DEEP_WIDE_WAVES
#define RT_DEEP_WIDE_WAVES 6
#endif
// The render loop; DEEP: the deep launch of a split pass (KParams::deep_mode),
// whose items are queued paths (no sample starts, no lens draws, no split) — its own
// instantiation, render_deep_kernel, so neither launch carries the other's code.
// WPB: waves per workgroup (4; the lone deep launch 8, which shares one LDS copy of the scene
// between twice the waves)
// PAIRS: the main launch of a pass that stores sample pairs (KParams::n_pair_items != 0,
// DESIGN.md §4.2), its own instantiation: the pair bookkeeping costs the loop ~3% of its issue
template <int V, int CULL, bool STATS, bool COUNT, bool DEEP, int WPB, bool PAIRS>
__device__ __forceinline__ void render_body(const KParams &p)
{
    constexpr bool FAST = (V == V_FAST_LDS);
    // Scene blob -> LDS (or read in place from global for the scalar-cache A/B variant):
    // [geo float4 x n_geo][sidx u32 x n_geo, 16-B padded][clusters float4 x 2 x n_clusters]
    extern __shared__ float4 lds_blob[];
    const float4 *blob;
    if constexpr (V == V_EXACT_SCALAR) {
        blob = p.blob;
    } else {
        for (uint32_t i = threadIdx.x; i < p.lds_units; i += blockDim.x) lds_blob[i] = p.blob[i];
        __syncthreads();
        blob = lds_blob;
    }
    // Per-render constants used only where a sample or an item starts are re-read from the
    // kernarg segment at each use (scalar loads) through a pointer made opaque every loop
    // iteration, so they do not pin ~30 SGPRs for the whole kernel (SGPR count bounds the
    // workgroups per CU on gfx950).
    typedef const __attribute__((address_space(4))) FrameConsts *fc_ptr_t;
    const fc_ptr_t fc_base =
        (fc_ptr_t)((const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr() +
                   offsetof(KParams, fc));
    typedef const __attribute__((address_space(4))) KParams *kp_ptr_t;
    const kp_ptr_t kp_base = (kp_ptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    const float4 *geo = blob;
    const uint32_t *sidx = reinterpret_cast<const uint32_t *>(blob + p.n_geo);
    const float4 *clus = blob + p.clus_offset;

    const uint32_t lane = threadIdx.x & 63u;
    // per-wave LDS of the transposed member tests
    TransposeLds *tw = nullptr;
    if constexpr (CULL == 7) {
        __shared__ TransposeLds s_tw[WPB];
        tw = &s_tw[threadIdx.x >> 6];
    }
    // per lane: a pending metal scatter's normal and roughness, or the geo entry {C, fl(r r)} of
    // the dielectric sphere the lane's path last hit (hint_candidate; its original index in lds_hid)
    __shared__ float4 lds_pn[64 * WPB];
    __shared__ uint32_t lds_hid[64 * WPB];
    __shared__ uint32_t lds_nb[64 * WPB];  // the dielectric sphere's shortcut word (hint_candidate)
    // (the lone deep kernel keeps the three in registers: RT_DEEP_REGHINT, an A/B build switch)
    constexpr bool kRegHint = DEEP && WPB == 8 && RT_DEEP_REGHINT;
    uint32_t r_hid = ~0u, r_nb = 0u;
    float4 r_pn = make_float4(0.f, 0.f, 0.f, 0.f);
    auto HID = [&](uint32_t sl) -> uint32_t & { if constexpr (kRegHint) return r_hid; else return lds_hid[sl]; };
    auto NB = [&](uint32_t sl) -> uint32_t & { if constexpr (kRegHint) return r_nb; else return lds_nb[sl]; };
    auto PN = [&](uint32_t sl) -> float4 & { if constexpr (kRegHint) return r_pn; else return lds_pn[sl]; };
    // sample pairs, per lane (structure of arrays): the main launch parks a pair's first colour
    // here while the lane traces the second (or, in word 0, the first's deep-queue index when it
    // went to the queue); the deep launch keeps the path's own queue index in word 0
    // (three words per lane for the pair's parked colour; one, the queue index, in the deep launch)
    __shared__ float lds_park[PAIRS ? 3 : 1][64 * WPB];
    auto park = [&](int c, uint32_t sl) -> float & { return lds_park[PAIRS ? c : 0][sl]; };
    const uint32_t wave_base = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);

    // the deep launch's waves issue ahead of other launches' waves (KParams::deep_prio): each of
    // its paths is a chain of ~56 dependent iterations, which beside other renders' waves on the
    // same SIMD would take ~7x as long
    if (DEEP && p.deep_prio) __builtin_amdgcn_s_setprio(3);
    // wave-uniform cursor over the item space (the deep launch: over the queued paths)
    // (the main launch: q / 8 is the item group the wave deals from, KParams::n_groups)
    uint32_t q = blockIdx.x & 7u, q_tried = 0;
    // static dealing (KParams::deep_static): this wave's next chunk of the deep queue, in the
    // order of the regions' chunks; the grid's waves take chunks w, w + waves, w + 2 waves, ...
    uint32_t deep_next = __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)WPB + (threadIdx.x >> 6));
    uint32_t cnext = 0, cend = 0;
    // the main launch: the chunk's items [cnext, run_end) lie in one sample, at slots run_base + ...
    uint32_t run_end = 0, run_base = 0;
    bool exhausted = false;

    // lane state: the lane's item is one sample (pixel enumeration index, sample of the pass)
    bool alive = false;
    // the main launch: it = the item word (rt_device.h kIt*); the deep launch: pix = the path's
    // slot, ls = its pair link
    uint32_t it = 0, pix = 0, ls = 0;
    f3 o = mk(0.f, 0.f, 0.f), d = o, att = o;
    uint32_t depth = 0;
    uint64_t rng = 0;
    // a lambert/metal hit leaves its scatter offset to the next iteration's rejection loop:
    // o = hit point; d = p + n (lambert) or reflect(unit(d), n) (metal); the metal's normal and
    // roughness wait in the lane's LDS word (pn: 16 B per lane, no registers held across the loop)
    bool pend = false, pend_metal = false;
    // a fresh sample whose lens draw did not finish within RT_REJECT_CAP attempts: its camera
    // stream state waits in (o.x, o.y) and its jittered (u, v) in (d.x, d.y) until it does
    bool pend_lens = false;
    // HID(lane) != ~0: the lane's last hit was a dielectric sphere, tested first next segment
    // (hint_candidate); kept in LDS, not in a register (at 72 VGPRs one more value spills)
    HID(thread_slot(wave_base)) = ~0u;
    // the instrumented kernel: neighbour words that no dielectric hit wrote point past any blob
    // (hint_candidate's bounds check)
    if (STATS) NB(thread_slot(wave_base)) = 0x3fffffffu;
    WaveTally<COUNT> wt;
    Dbg dbg{};
    uint32_t dbg_iters = 0, dbg_refills = 0, dbg_iters_dry = 0, dbg_dealt = 0, dbg_walks = 0;
    uint32_t dbg_walks_nohint = 0;  // (deep launch) walks with a walking lane that has no hint sphere
    uint64_t t_dry = 0;  // STATS: realtime when this wave found every queue empty
    // STATS build only: shader-clock cycles per loop region, summed over the wave's iterations
    uint64_t cyc[5] = {0, 0, 0, 0, 0};  // refill, sample start, closest hit, shading, fold
    uint64_t t_prev = STATS ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t t_wave0 = STATS ? __builtin_amdgcn_s_memrealtime() : 0;  // 100 MHz clock
    auto stamp = [&](int r) {
        if (STATS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            cyc[r] += t - t_prev;
            t_prev = t;
        }
    };

    for (;;) {
        stamp(4);
#ifdef RT_EXTRA_VALU  // timing probe only (scripts/build_variant.sh): RT_EXTRA_VALU more VALU per wave iteration
        {
            float e0 = o.x, e1 = o.y, e2 = o.z, e3 = d.x;
            asm volatile("" : "+v"(e0), "+v"(e1), "+v"(e2), "+v"(e3));
#pragma unroll
            for (int k = 0; k < RT_EXTRA_VALU / 4; ++k) {
                e0 = fmaf(e0, 1.0001f, 0.5f); e1 = fmaf(e1, 1.0001f, 0.5f);
                e2 = fmaf(e2, 1.0001f, 0.5f); e3 = fmaf(e3, 1.0001f, 0.5f);
            }
            asm volatile("" ::"v"(e0), "v"(e1), "v"(e2), "v"(e3));
        }
#endif
#ifdef RT_EXTRA_SALU  // timing probe only: RT_EXTRA_SALU more SALU per wave iteration
        {
            uint32_t s0 = __builtin_amdgcn_readfirstlane(pix);
#pragma unroll
            for (int k = 0; k < RT_EXTRA_SALU; ++k) asm volatile("s_add_u32 %0, %0, 3" : "+s"(s0));
            asm volatile("" ::"s"(s0));
        }
#endif
        fc_ptr_t fc = fc_base;
#if RT_DEEP_HOIST
        if (!(DEEP && WPB == 8))
#endif
        asm volatile("" : "+s"(fc));
        // the kernel parameters, re-read from the kernarg segment each iteration through an
        // opaque pointer: their uses (the deep split, the shading records, the refill) then
        // hold no SGPRs across the loop (31 SGPRs were spilled to VGPR lanes otherwise)
        kp_ptr_t kpp = kp_base;
#if RT_DEEP_HOIST
        if (!(DEEP && WPB == 8))
#endif
        asm volatile("" : "+s"(kpp));
        const __attribute__((address_space(4))) KParams &P = *kpp;
        // ---- refill items for idle lanes and start their samples -------------------
        uint64_t need = ballot(!alive);
        bool fresh = false;
        if (STATS && need && !exhausted && lane == 0) ++dbg_refills;
        while (need && !exhausted) {
            RT_EV(EV_REFILL_TRIP);
            // (the main launch: run_end <= cend, so a finished chunk is a finished run)
            if (DEEP ? cnext >= cend : cnext >= run_end) {
            if (cnext >= cend) {
                uint32_t c = 0;
                if constexpr (DEEP) {
                    if (WPB == 8 && P.deep_static) {  // (the lone deep launch's instantiation only)
                        // the regions' path counts are final (the main launch has ended): lanes
                        // 0-7 read them in one round trip; chunk j of the concatenated regions
                        // goes to wave j mod waves. No atomics: thousands of waves probing eight
                        // shared counters at the end of a launch cost more than the paths
                        const uint32_t n = lane < 8u ? min(P.deep.ctr[lane * kQueueStride + kDeepCount], P.deep.rcap) : 0u;
                        const uint32_t j = deep_next;
                        deep_next += gridDim.x * (uint32_t)WPB;
                        // lane k < 8: region k's chunks and their first index (exclusive prefix
                        // over lanes 0..k-1, three shuffle steps); the region holding chunk j
                        const uint32_t ck = (n + 63u) / 64u;
                        uint32_t incl = ck;
#pragma unroll
                        for (uint32_t off = 1; off < 8u; off <<= 1) {
                            const uint32_t v = (uint32_t)__shfl_up((int)incl, off);
                            if (lane >= off) incl += v;
                        }
                        const uint64_t hit = ballot(lane < 8u && j < incl && j >= incl - ck);
                        if (!hit) {
                            exhausted = true;
                            continue;
                        }
                        const uint32_t r = (uint32_t)__builtin_ctzll(hit);
                        const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)(incl - ck), (int)r);
                        const uint32_t nr = (uint32_t)__builtin_amdgcn_readlane((int)n, (int)r);
                        cnext = r * P.deep.rcap + 64u * (j - base);
                        cend = r * P.deep.rcap + min(64u * (j - base) + 64u, nr);
                        goto deal;
                    }
                    // the deep launch: 64 queued paths per grab from region q, then the next
                    // region (a wave starts on its workgroup's region)
                    if (lane == 0) c = atomicAdd(P.deep.ctr + q * kQueueStride + kDeepDeal, 1u);
                    c = __builtin_amdgcn_readfirstlane(c);
                    const uint32_t nq = __builtin_amdgcn_readfirstlane(
                        min(P.deep.ctr[q * kQueueStride + kDeepCount], P.deep.rcap));
                    if (c >= (nq + 63u) / 64u) {
                        q = (q + 1u) & 7u;
                        if (++q_tried == 8u) exhausted = true;
                        continue;
                    }
                    cnext = __builtin_amdgcn_readfirstlane(q * P.deep.rcap + 64u * c);
                    cend = __builtin_amdgcn_readfirstlane(q * P.deep.rcap + min(64u * c + 64u, nq));
                } else {
                const uint32_t grp = q >> 3, qq = q & 7u;
                if (lane == 0) c = atomicAdd(P.queue_ctr + qq * kQueueStride + grp, 1u);  // word grp of queue qq's line
                c = __builtin_amdgcn_readfirstlane(c);
                // guided: queue q owns blocks [qb0, qb1) of 64 items of the group (group-local
                // indices, KParams::n_groups); ticket c takes blocks
                // [S(c), S(c+1)), S(t) = min(B, floor(B (1 - beta^t)) + 2t): chunks shrink
                // geometrically from ~B / (K waves per queue) to 2 blocks, so a queue is
                // served by few atomics and its last chunks are small. S is the same
                // function for every wave, so consecutive tickets tile the range; the 2t
                // term keeps it increasing even if exp2 or the float product is off by an
                // ulp (one block at most).
                const uint32_t GB = grp == 0u ? P.grp_blocks[0] : grp == 1u ? P.grp_blocks[1] : P.grp_blocks[2];
                const uint32_t qb0 = (uint32_t)(((uint64_t)GB * qq) >> 3);
                const uint32_t B = (uint32_t)(((uint64_t)GB * (qq + 1u)) >> 3) - qb0;
                auto S = [&](uint32_t t) -> uint32_t {
                    const float x = t ? exp2f((float)t * P.guided_l2b) : 1.f;
                    const uint64_t g = (uint64_t)floorf((float)B * (1.f - x)) + 2ull * t;
                    return g < B ? (uint32_t)g : B;
                };
                const uint32_t s0 = __builtin_amdgcn_readfirstlane(S(c));
                if (s0 >= B) {
                    // the group's next queue; after all 8, the next group (a group is dealt
                    // whole, by every wave, before the next one starts)
                    q = (q & ~7u) | ((q + 1u) & 7u);
                    if (++q_tried == 8u) {
                        q_tried = 0;
                        q += 8u;
                        if (q >= 8u * P.n_groups) exhausted = true;
                    }
                    continue;
                }
                const uint32_t GI = grp == 0u ? P.grp_items[0] : grp == 1u ? P.grp_items[1] : P.grp_items[2];
                cnext = 64u * (qb0 + s0);
                cend = __builtin_amdgcn_readfirstlane(min(64u * (qb0 + S(c + 1u)), GI));
                }
            }
            if constexpr (!DEEP) {
                // the chunk's run within one sample: group grp's item J is sample J / ng at
                // position p0 + J % ng, slot [sample][position] (sample-major over the pass's
                // permuted enumeration); one group (natural order): slot J
                const uint32_t grp = q >> 3;
                const uint32_t p0 = grp == 0u ? 0u : grp == 1u ? P.grp_pix[1] : P.grp_pix[2];
                const uint32_t ng = (grp == 0u ? P.grp_pix[1] : grp == 1u ? P.grp_pix[2] : P.grp_pix[3]) - p0;
                UDiv dv;
                dv.m = grp == 0u ? P.div_grp[0].m : grp == 1u ? P.div_grp[1].m : P.div_grp[2].m;
                dv.s1 = grp == 0u ? P.div_grp[0].s1 : grp == 1u ? P.div_grp[1].s1 : P.div_grp[2].s1;
                dv.s2 = grp == 0u ? P.div_grp[0].s2 : grp == 1u ? P.div_grp[1].s2 : P.div_grp[2].s2;
                const uint32_t sj = __builtin_amdgcn_readfirstlane(udiv(cnext, dv));
                run_end = __builtin_amdgcn_readfirstlane(min(cend, (sj + 1u) * ng));
                run_base = __builtin_amdgcn_readfirstlane(sj * P.n_pixels + p0 + (cnext - sj * ng));
            }
            }
        deal:
            const uint32_t avail = (DEEP ? cend : run_end) - cnext;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            if (!alive && rank < avail) {
                uint32_t I = (DEEP ? cnext : run_base) + rank;
                if constexpr (DEEP) {
                    // a queued path resumes where the main launch left it: the ray of its next
                    // segment, attenuation, data stream and segment count; ls = 0 and pix = the
                    // slot index address the same slot
                    const uint32_t cap = 8u * P.deep.rcap;
                    I = checked<STATS>(I, cap, BC_DEEP_ITEM, p.dbg);
                    const float *f = P.deep.f;
                    o = mk(f[I], f[cap + I], f[2 * cap + I]);
                    d = mk(f[3 * cap + I], f[4 * cap + I], f[5 * cap + I]);
                    att = mk(f[6 * cap + I], f[7 * cap + I], f[8 * cap + I]);
                    rng = P.deep.rng[I];
                    pix = P.deep.slot[I];
                    ls = P.deep.link[I];  // the deep launch: ls is the path's pair link
                    depth = P.deep_mode;
                    alive = true;
                    // its hint sphere (hint_candidate): the geo entry from the shading record
                    const uint32_t hid = P.deep.hid[I], sl = thread_slot(wave_base);
                    lds_park[0][sl] = __uint_as_float(I);
                    if (hid != ~0u) {
                        // (from LDS when the launch staged the shading records there: a lone
                        // deep launch, whose refills then wait on no second global round trip)
                        const uint32_t ib = checked<STATS>(hid & 0x7fffffffu, P.n_spheres, BC_DEEP_HINT, p.dbg);
                        const uint32_t di = P.shade_offset + 2 * P.n_spheres + (P.n_spheres + 15u) / 16u + ib;
                        float4 sf, dr;
                        if (P.shade_lds) {
                            sf = blob[P.shade_offset + 2u * ib];
                            dr = blob[di];
                            asm volatile("");
                        } else {
                            sf = gld4(P.blob + P.shade_offset, 2u * ib);
                            dr = gld4(P.blob, di);
                        }
                        PN(sl) = make_float4(sf.x, sf.y, sf.z, sf.w * sf.w);
                        NB(sl) = __float_as_uint(dr.w);
                    }
                    HID(sl) = hid;
                } else {
                    it = I;  // a pair item (the pass's full blocks) or a single tail sample; its slot
                    alive = fresh = true;
                }
            }
            const uint32_t took = min((uint32_t)__popcll(need), avail);
            if (STATS) dbg_dealt += took;
            cnext += took;
            if (!DEEP) run_base += took;
            need = ballot(!alive);
        }

        // a pair whose first sample ended last iteration: its second sample starts now
        if (!DEEP && PAIRS && (it & kItRestart)) {
            fresh = true;
            it &= ~kItRestart;
        }
        stamp(0);
        // ---- start the sample of a freshly assigned item (main.cxx:192-200) -----------
        const uint64_t inc_data = ((uint64_t)fc->inc_data_hi << 32) | fc->inc_data_lo;
        // A sample's colour is final (main.cxx:205 sums it): a single's goes to its slot; a pair's
        // first is parked in the lane's scratch word and its second sample starts next iteration
        // (true: the lane sits out the rest of this one); the second's completes the pair sum
        // RN(c_2j + c_2j+1) in the pair's slot. In the deep launch the path's pair link says where
        // its partner's colour is.
        // the pixel (enumeration index) and the sample of the pass of the lane's item word
        auto item_pixel = [&](uint32_t &s) -> uint32_t {
            const uint32_t sl = it & kItSlot;
            const uint32_t npi = PAIRS ? (uint32_t)P.n_pair_items : 0u;
            const bool pr = sl < npi;
            const uint32_t J = pr ? sl : sl - npi;
            const uint32_t q = udiv(J, fc->div_n_pixels);
            s = !PAIRS ? q : pr ? 2u * q + (it >> 31) : 2u * fc->n_pairs + q;
            return J - q * fc->n_pixels;
        };
        auto finish = [&](f3 col) -> bool {
            float *dst;
            if constexpr (DEEP) {
                const uint32_t role = ls >> 30;
                dst = P.slots + (size_t)checked<STATS>(pix, P.n_slots, BC_SLOT, p.dbg) * 3u;
                if (role == kRolePartnerDone) {
                    // the partner ended in the main launch and left its colour in the slot
                    // (IEEE addition is commutative: the order of the pair's two terms is moot)
                    col = mk(dst[0], dst[1], dst[2]) + col;
                } else if (role != kRoleSingle) {
                    // both samples of the pair came here: the second of the two to end sums.
                    // Each leaves its colour in its own entry (its o.xyz words, read at its
                    // refill) with device-scope atomics, then counts its arrival at the first's
                    // entry; the one that finds the other arrived reads that colour back with
                    // atomics (device-scope atomics are coherent across the XCDs' L2s)
                    const uint32_t cap = 8u * P.deep.rcap, self = __float_as_uint(lds_park[0][thread_slot(wave_base)]);
                    const uint32_t partner = ls & kLinkIndex, first = role == kRoleBothFirst ? self : partner;
                    uint32_t *fw = reinterpret_cast<uint32_t *>(P.deep.f);
                    const uint32_t r = atomicExch(fw + self, __float_as_uint(col.x)) ^
                                       atomicExch(fw + cap + self, __float_as_uint(col.y)) ^
                                       atomicExch(fw + 2u * cap + self, __float_as_uint(col.z));
                    uint32_t one = 1u;
                    asm volatile("" : "+v"(one) : "v"(r));  // the arrival after the colour is stored
                    if (atomicAdd(P.deep.meet + first, one) != 1u) {
                        alive = false;  // the partner has not ended: it sums
                        return false;
                    }
                    const f3 cp = mk(__uint_as_float(atomicOr(fw + partner, 0u)), __uint_as_float(atomicOr(fw + cap + partner, 0u)),
                                     __uint_as_float(atomicOr(fw + 2u * cap + partner, 0u)));
                    col = role == kRoleBothFirst ? col + cp : cp + col;  // RN(c_2j + c_2j+1)
                    if (STATS) ++dbg.ev[EV_BOTH_MEET];
                    atomicExch(P.deep.meet + first, 0u);               // zero again for the next pass
                }
            } else {
                const uint32_t slot = it & kItSlot;
                if (PAIRS && slot < P.n_pair_items) {
                    const uint32_t sl = thread_slot(wave_base);
                    if (!(it & kItSecond)) {
                        park(0, sl) = col.x;
                        park(1, sl) = col.y;
                        park(2, sl) = col.z;
                        it |= kItSecond | kItRestart;
                        return true;
                    }
                    // the first's colour, unless it went to the deep queue (which then adds this one)
                    if (!(it & kItFirstDeep)) {
                        col = mk(park(0, sl), park(1, sl), park(2, sl)) + col;  // RN(c_2j + c_2j+1)
                        if (STATS) ++dbg.ev[EV_PAIR_SUM];
                    }
                }
                dst = P.slots + (size_t)checked<STATS>(slot, P.n_slots, BC_SLOT, p.dbg) * 3u;  // < 2^29: one pass holds <= 2 GiB of slots
            }
            dst[0] = col.x;
            dst[1] = col.y;
            dst[2] = col.z;
            alive = false;
            return false;
        };
        uint64_t rc = 0;  // the camera stream of a fresh sample
        float uu = 0.f, vv = 0.f;
        if (fresh) {
            RT_EV(EV_FRESH);
            uint32_t px, rr, ls;
            pixel_of(*fc, item_pixel(ls), px, rr, P.block_perm);
            const uint32_t py = fc->row_offset + rr * fc->row_stride;
            const uint32_t s = fc->sample_begin + ls;
            // key = (y W + x) spp + s (y W + x < 2^32: the host bounds W H)
            const uint64_t key = (uint64_t)(py * fc->W + px) * fc->spp + s;
            const uint64_t inc_cam = ((uint64_t)fc->inc_cam_hi << 32) | fc->inc_cam_lo;
            // pcg_seed(key, inc) = (inc + key) M + inc = key M + inc (M + 1): one vector multiply
            // for both streams, the inc (M + 1) terms are wave-uniform (scalar)
            const uint64_t km = key * kPcgMul;
            rng = km + inc_data * (kPcgMul + 1u);
            rc = km + inc_cam * (kPcgMul + 1u);
            const float fW = fc->fW, fH = fc->fH, rW = fc->rW, rH = fc->rH;
            const uint32_t df = fc->div_fast;
            const float xu = canonical(rng, inc_data);  // the u jitter's draw, then v's
            const float xv = canonical(rng, inc_data);
            if (df == 3u) {
                // both divisors take the checked short form (the common case): one uniform
                // branch for the four divisions instead of one per division
                uu = div_const((float)px, fW, rW, true) + div_const(xu, fW, rW, true);
                vv = div_const((float)py, fH, rH, true) + div_const(xv, fH, rH, true);
            } else {
                const bool fw = df & 1u, fh = df & 2u;
                uu = div_const((float)px, fW, rW, fw) + div_const(xu, fW, rW, fw);
                vv = div_const((float)py, fH, rH, fh) + div_const(xv, fH, rH, fh);
            }
            att = mk(1.f, 1.f, 1.f);
            depth = 0;
            HID(thread_slot(wave_base)) = ~0u;
        }
        // ---- one rejection loop for the wave (raytracer.hxx:32-43) ------------------------
        // Fresh lanes draw the lens offset from their camera stream (camera.hxx:52); lanes
        // whose last hit was lambert or metal draw their scatter offset from their data stream
        // (raytracer.hxx:135,147). Serving both in ONE loop makes the wave pay the longest
        // rejection run of the union of those lanes once per iteration instead of once per
        // kind; every stream still sees exactly its own draws in its own order.
        // A lane whose draws are not accepted within RT_REJECT_CAP attempts sits this iteration
        // out (`defer`) and resumes its own draw sequence in the next one: the wave no longer
        // waits for its unluckiest lane's whole run (mean 1.91 attempts, ~6.9 for the worst of
        // 64 lanes), and every stream still sees the same draws in the same order.
        bool defer = false;
        bool absorbed = false;  // a metal scatter absorbed: colour 0, finished at the iteration's end

        const bool lens = !DEEP && (fresh || pend_lens);
        if (lens || pend) {
            const uint64_t inc = lens ? (((uint64_t)fc->inc_cam_hi << 32) | fc->inc_cam_lo) : inc_data;
            if (pend_lens) {
                uu = d.x;
                vv = d.y;
                rc = ((uint64_t)__float_as_uint(o.y) << 32) | __float_as_uint(o.x);
            }
            uint64_t st = lens ? rc : rng;
            bool got;
            const f3 r = random_in_unit_sphere_capped<STATS>(st, inc, got, dbg);
            if (!got) {
                defer = true;
                if (lens) {
                    pend_lens = true;
                    o.x = __uint_as_float((uint32_t)st);
                    o.y = __uint_as_float((uint32_t)(st >> 32));
                    d.x = uu;
                    d.y = vv;
                } else {
                    rng = st;  // pend stays set
                }
            } else if (lens) {
                RT_EV(EV_LENS_DONE);
                pend_lens = false;
                // camera.hxx:46-57
                const f3 rd = r * fc->lens;
                const f3 off = mk(uu * rd.x, vv * rd.y, 0.f);
                const f3 org = mk(fc->org[0], fc->org[1], fc->org[2]);
                o = org + off;
                d = ((mk(fc->llc[0], fc->llc[1], fc->llc[2]) + mk(fc->hor[0], fc->hor[1], fc->hor[2]) * uu) +
                     mk(fc->ver[0], fc->ver[1], fc->ver[2]) * (1.f - vv)) - off;
                if (fc->corrected) d = d - org;
            } else {
                RT_EV(EV_SCATTER_DONE);
                rng = st;
                if (!pend_metal) {
                    d = (d + r) - o;                       // lambert :135, d held p + n, o = p
                } else {
                    const float4 pn = PN(thread_slot(wave_base));
                    const f3 nd = d + r * pn.w;            // metal :147, d held reflect(unit(d), n)
                    if (dot(nd, mk(pn.x, pn.y, pn.z)) > 0.f) {
                        d = nd;
                    } else {                               // absorbed: main.cxx:68, colour 0
                        RT_EV(EV_METAL_ABSORB);
                        absorbed = defer = true;  // it traces nothing more
                    }
                }
                pend = false;
            }
        }
        stamp(1);
        // no live lane: the wave's refill found the item space exhausted (a metal path absorbed
        // above stays alive until finish() stores its colour at the end of this iteration)
        if (ballot(alive) == 0) {
            if (exhausted) break;
            continue;
        }
        // ---- deep-path split: a path that has traced deep_depth segments (with its scatter
        // resolved) moves to the deep queue, whole state, and the lane takes a new item next
        // iteration. The few paths that run to max_depth (the reference's refract traps rays in
        // glass spheres) then no longer hold this launch's waves for ~max_depth iterations after
        // the item queues run dry; the deep launch runs them with every lane busy. Each path
        // sees the same operations and draws in the same order: same bits.
        // A path goes to region (its dielectric sphere's index) % 8 of the queue, or
        // blockIdx % 8 if its last hit was not dielectric: the paths trapped in one sphere then
        // share a region, and the deep launch's waves, which deal 64 paths at a time from one
        // region, trace paths of the same few spheres, whose segments reach the same few
        // clusters (8 counters on separate lines spread the appends). A path that finds its
        // region full stays in this launch.
        if (!DEEP && P.deep_depth) {
            const bool dv = alive && !defer && depth == P.deep_depth;
            if (ballot(dv)) {
                uint32_t j = ~0u, r = 0;
                if (dv) {
                    const uint32_t hid = HID(thread_slot(wave_base));
                    r = hid != ~0u ? (hid & 7u) : (blockIdx.x & 7u);
                    j = atomicAdd(P.deep.ctr + r * kQueueStride + kDeepCount, 1u);
                }
                if (dv && j < P.deep.rcap) {
                    const uint32_t cap = 8u * P.deep.rcap;
                    j = checked<STATS>(j + r * P.deep.rcap, cap, BC_DEEP_APPEND, p.dbg);
                    uint32_t ss;
                    const uint32_t px = checked<STATS>(item_pixel(ss), fc->n_pixels, BC_DEEP_PX, p.dbg);
                    float *f = P.deep.f;
                    f[j] = o.x; f[cap + j] = o.y; f[2 * cap + j] = o.z;
                    f[3 * cap + j] = d.x; f[4 * cap + j] = d.y; f[5 * cap + j] = d.z;
                    f[6 * cap + j] = att.x; f[7 * cap + j] = att.y; f[8 * cap + j] = att.z;
                    P.deep.rng[j] = rng;
                    P.deep.hid[j] = HID(thread_slot(wave_base));
                    P.deep.px[px] = 1;
                    // the path's slot and pair link (rt_device.h kRole*)
                    const uint32_t slot = it & kItSlot, sl = thread_slot(wave_base);
                    uint32_t link = kRoleSingle << 30;
                    if (!PAIRS || slot >= P.n_pair_items) {
                        alive = false;
                    } else {
                        link = kRolePartnerDone << 30;
                        if (!(it & kItSecond)) {
                            // the pair's first: the lane traces the second next iteration, which
                            // leaves its colour in the slot (or joins this one in the queue)
                            lds_park[0][sl] = __uint_as_float(j);
                            it |= kItSecond | kItFirstDeep | kItRestart;
                            defer = true;  // sits out the rest of this iteration
                        } else {
                            if (it & kItFirstDeep) {  // both of the pair queued: they meet there
                                const uint32_t j1 = __float_as_uint(lds_park[0][sl]);
                                link = (kRoleBothSecond << 30) | j1;
                                P.deep.link[j1] = (kRoleBothFirst << 30) | j;
                            } else {  // the first's colour, parked in the lane's LDS words, to the slot
                                float *dst = P.slots + (size_t)checked<STATS>(slot, P.n_slots, BC_SLOT, p.dbg) * 3u;
                                dst[0] = park(0, sl);
                                dst[1] = park(1, sl);
                                dst[2] = park(2, sl);
                            }
                            alive = false;
                        }
                    }
                    P.deep.slot[j] = slot;
                    P.deep.link[j] = link;
                }
            }
        }
        RT_EV(EV_ITER);
        if (STATS) {
            const uint32_t nl = lanes(alive);
            if (first_active_lane()) {
                dbg.ev[EV_LIVE_LANES] += nl;
                if (exhausted) {
                    ++dbg.ev[EV_DRY_ITER];
                    dbg.ev[EV_DRY_LANES] += nl;
                }
            }
        }
        if (STATS && lane == 0) {
            ++dbg_iters;
            if (exhausted) {
                if (!dbg_iters_dry) t_dry = __builtin_amdgcn_s_memrealtime();
                ++dbg_iters_dry;
            }
        }

        // ---- closest hit of one segment for every live lane -----------------------------
        const bool seg = alive && !defer && depth < P.max_depth;  // depth check: main.cxx:74
        // |d|^2 (raytracer.hxx:56) and its refined reciprocal for this segment's roots; the sky
        // below reuses both (unit_direction's length is sqrt of the same sum)
        const float a = d.x * d.x + d.y * d.y + d.z * d.z;
        const uint64_t segm = ballot(seg);
        const RayDiv rd = ray_div(a, segm, P.fast_roots);
        Hit h{kNoHit};
        if constexpr (CULL == 7) {  // whole wave: every lane helps with transposed member tests
            uint64_t key0 = no_hit();
            bool skip = false;
            const uint32_t sl = thread_slot(wave_base);
            const uint32_t hid = HID(sl);
            if (ballot(seg && hid != ~0u))
                key0 = hint_candidate<FAST, STATS>(seg && hid != ~0u, PN(sl), hid, NB(sl), geo, sidx, o, d, rd, P.iso,
                                                   skip, P.n_geo, P.diag_unbounded_nb, p.dbg);
            const bool walk = seg && !skip;
            const uint64_t wm = ballot(walk);
            if (STATS && first_active_lane()) {
                dbg.ev[EV_ISO_LANES] += (uint32_t)__popcll(segm & ~wm);
                if (segm && !wm) ++dbg.ev[EV_WALK_SKIPPED];
                const uint32_t nw = (uint32_t)__popcll(wm);
                if (nw == 1u) ++dbg.ev[EV_WALK1];
                else if (nw == 2u) ++dbg.ev[EV_WALK2];
                else if (nw >= 3u && nw <= 4u) ++dbg.ev[EV_WALK4];
                else if (nw >= 5u && nw <= 8u) ++dbg.ev[EV_WALK8];
            }
            if (STATS) {
                const uint64_t nh = ballot(walk && hid == ~0u);
                if (lane == 0 && wm) ++dbg_walks;  // iterations in which the wave walked
                if (lane == 0 && nh) ++dbg_walks_nohint;
            }
            h = closest_hit<FAST, CULL, STATS, COUNT>(P, geo, sidx, clus, o, d, rd, dbg, wt, walk, wm, tw, key0);
            if (!seg) h = Hit{kNoHit};
        } else if (seg) {
            h = closest_hit<FAST, CULL, STATS, COUNT>(P, geo, sidx, clus, o, d, rd, dbg, wt, true, segm, nullptr, no_hit());
        }
        stamp(2);
        {
            const uint32_t ns = lanes(seg);  // segments of this iteration (main.cxx:74 passed)
            wt.add_seg(ns);
            wt.add_sph((uint64_t)ns * P.n_always);
        }

        // ---- shading: the hit of every live lane -----------------------------------------
        bool done = absorbed;
        f3 col = mk(0.f, 0.f, 0.f);
        if (alive && !defer) {
            if (!seg) {
                done = true;  // main.cxx:74 (only reachable with max_depth == 0)
            } else {
                const float t = h.t();
                uint32_t ib = h.id();
                ++depth;
                if (ib == 0xffffffffu) {
                    RT_EV(EV_SKY);
                    // main.cxx:71: background(.5 * unit_direction.y + 1) * attenuation. With the
                    // short forms (rd.fd: a in [2^-40, 2^40]) the length is sqrt_scaled(a) >= 2^-20
                    // and d.y / length is exact unless |d.y| < 2^-100, where both forms give
                    // |y| < 2^-80 and tt rounds to 1 either way.
                    float uy;
                    if (rd.fd != 0u) {
                        const float l = sqrt_scaled(a);
                        const float y0 = __builtin_amdgcn_rcpf(l);
                        uy = div_ray(d.y, RayDiv{l, fmaf(fmaf(-l, y0, 1.f), y0, y0), true});
                    } else {
                        uy = normalize(d).y;
                    }
                    const float tt = .5f * uy + 1.f;
                    const f3 bg = mk(1.f, 1.f, 1.f) * (1.f - tt) + mk(.5f, .7f, 1.f) * tt;
                    col = bg * att;
                    done = true;
                } else if (depth >= P.max_depth) {
                    // main.cxx:65-74: a scattered ray would not be traced and an absorbed one
                    // returns 0 too; this sample's streams are not drawn from again
                    done = true;
                } else {
                    RT_EV(EV_HIT);
                    ib = checked<STATS>(ib, P.n_spheres, BC_SHADE, p.dbg);
                    float4 sf, md;
                    uint32_t kind;
                    if (V != V_EXACT_SCALAR && P.shade_lds) {
                        const float4 *shade = blob + P.shade_offset;
                        sf = shade[2 * ib];
                        md = shade[2 * ib + 1];
                        kind = reinterpret_cast<const uint8_t *>(shade + 2 * P.n_spheres)[ib];
                        asm volatile("");  // keeps the LDS and global loads apart (no sinking)
                    } else {
                        // global memory, named as such: the two branches' loads would otherwise be
                        // merged into flat loads through a selected pointer
                        const float4 *shade = P.blob + P.shade_offset;
                        sf = gld4(shade, 2 * ib);
                        md = gld4(shade, 2 * ib + 1);
                        kind = ((const __attribute__((address_space(1))) uint8_t *)(shade + 2 * P.n_spheres))[ib];
                    }
                    const f3 ctr = mk(sf.x, sf.y, sf.z);
                    const f3 hp = o + d * t;                    // ray::point_at, math.hxx:353
                    // raytracer.hxx:71. With the scene in the short-form range (|r| in [2^-40, 2^19],
                    // P.fast_roots) the division by r takes the short form unless a lane's offset has
                    // a component below 2^-100 (zero included).
                    const f3 dv = hp - ctr;
                    f3 hn;
                    if (P.fast_roots && all_lanes_min_abs_ok(dv)) hn = div3_short(dv, sf.w);
                    else hn = dv / sf.w;
                    att = att * mk(md.x, md.y, md.z);           // main.cxx:65 (unused if absorbed)
                    // raytracer.hxx:120-199
                    o = hp;
                    if (kind != 2u) HID(thread_slot(wave_base)) = ~0u;  // no hint after lambert, metal
                    if (kind == 0u) {                           // lambert, :132-141
                        RT_EV(EV_LAMBERT);
                        d = hp + hn;                            // + rius next iteration, then - p
                        pend = true;
                        pend_metal = false;
                    } else {
                        // metal and dielectric lanes share one unit direction and one reflection
                        // (one code path for the wave instead of two)
                        RT_EV(EV_UNIT_DIR);
                        // unit_vector(d) (math.hxx:219-227): length sqrt(a) with a = |d|^2 as above;
                        // under rd.fd, a in [2^-40, 2^40], so the length is sqrt_scaled(a) in
                        // [2^-20, 2^20] and the three divisions take the short form unless a
                        // lane's direction has a component below 2^-100
                        f3 ud;
                        if (rd.fd != 0u && all_lanes_min_abs_ok(d)) ud = div3_short(d, sqrt_scaled(a));
                        else ud = normalize(d);
                        const f3 rf = reflect(ud, hn);
                        if (kind == 1u) {                       // metal, :143-156
                            d = rf;                             // + rius * roughness next iteration
                            PN(thread_slot(wave_base)) = make_float4(hn.x, hn.y, hn.z, md.w);
                            pend = true;
                            pend_metal = true;
                        } else {                                // dielectric, :158-194
                            RT_EV(EV_DIELECTRIC);
                            // {1 / ior, x(ior), x(1 / ior), shortcut word} of this sphere, x(r) = (1 - r) / (1 + r)
                            const float4 dcs = dielectric_record<V>(P, blob, ib);
                            {   // the next segment tests this sphere first (hint_candidate)
                                const uint32_t sl = thread_slot(wave_base);
                                PN(sl) = make_float4(sf.x, sf.y, sf.z, sf.w * sf.w);  // its geo entry, raytracer.hxx:58
                                const uint32_t w = __float_as_uint(dcs.w);  // its shortcut word
                                HID(sl) = ib | (w & kShortcut);
                                NB(sl) = w;
                            }
                            f3 outward = mk(-hn.x, -hn.y, -hn.z);
                            float ri = md.w, xs = dcs.y;
                            float cosv = dot(ud, hn);
                            if (cosv <= 0.f) {
                                outward = outward * -1.f;
                                ri = dcs.x;                     // 1.f / ri
                                xs = dcs.z;
                                cosv *= -1.f;
                            }
                            const f3 refr = refract(ud, outward, ri);
                            float prob = 1.f;
                            // length(refr) > 0 <=> norm > 0 (correctly rounded sqrt; NaN -> false)
                            if (refr.x * refr.x + refr.y * refr.y + refr.z * refr.z > 0.f) prob = schlick_x(xs, cosv);
                            d = canonical(rng, inc_data) < prob ? rf : refr;
                        }
                    }
                }
            }
            stamp(3);
        }
        if (done) {
            RT_EV(EV_STORE);
            // the sample's colour goes to its slot or its pair; accumulate_kernel forms the
            // reference's blocked sum over the slots (main.cxx:205)
            finish(col);
        }
    }

    if (COUNT && p.segments) {
        // wave reductions, one atomic per wave and counter: [0] segments, [1] sphere tests,
        // [2] cluster box tests (lane-level, executed)
        if (lane == 0) {  // one atomic per wave and counter
            atomicAdd(p.segments + 0, (unsigned long long)wt.seg);
            atomicAdd(p.segments + 1, (unsigned long long)wt.sph);
            atomicAdd(p.segments + 2, (unsigned long long)wt.box);
        }
    }
    if (STATS && p.dbg) {
        const uint32_t c[8] = {dbg_iters, dbg_refills, dbg.wave_blocks, dbg.lane_blocks, dbg.wave_roots,
                               dbg.lane_roots, lane == 0 ? (uint32_t)wt.seg : 0u, dbg.wave_member_blocks};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned long long v = c[i];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(p.dbg + i, v);
        }
#pragma unroll
        for (int i = 0; i < (int)EV_COUNT; ++i) {
            unsigned long long v = dbg.ev[i];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(p.dbg + kDbgEvBase + i, v);
        }
        if (lane == 0) {
            for (int i = 0; i < 5; ++i) atomicAdd(p.dbg + 8 + i, (unsigned long long)cyc[i]);
            atomicMax(p.dbg + 14, ~t_wave0);  // launch start = ~max(~t) = earliest wave start
            atomicAdd(p.dbg + 13, (unsigned long long)dbg_dealt);  // items (deep: paths) dealt
        }
        // wave timeline: [16 + 4w] time the queues were found dry (realtime ticks), [17 + 4w] exit,
        // [18 + 4w] shader-clock cycles in the loop << 32 | refill rounds << 16 | loop iterations,
        // [19 + 4w] hardware id << 48 | iterations after dry << 32 | the wave's start (low 32 bits of
        // the realtime clock); w = wave of the grid. The launch starts at t_wave0 of the earliest wave.
        const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (lane == 0 && w < kDbgWaves) {
            const unsigned long long cy = cyc[0] + cyc[1] + cyc[2] + cyc[3] + cyc[4];
            // (a deep launch: the walks with a lane that has no hint sphere << 32 | the walks)
            p.dbg[16 + 4 * w] = DEEP ? ((unsigned long long)dbg_walks_nohint << 32 | dbg_walks)
                                     : (t_dry ? t_dry : __builtin_amdgcn_s_memrealtime());
            p.dbg[17 + 4 * w] = __builtin_amdgcn_s_memrealtime();
            p.dbg[18 + 4 * w] = (min(cy, 0xffffffffull) << 32) | (min(dbg_refills, 65535u) << 16) | min(dbg_iters, 65535u);
            p.dbg[19 + 4 * w] = ((unsigned long long)(__smid() & 0xffffu) << 48) |
                                ((unsigned long long)min(DEEP ? dbg_walks : dbg_iters_dry, 65535u) << 32) | (uint32_t)t_wave0;
        }
    }
}

template <int V, int CULL, bool STATS, bool COUNT, bool PAIRS = false>
__global__ __launch_bounds__(256, (kMinWaves<V, CULL, STATS>)) void render_kernel(const KParams p)
{
    render_body<V, CULL, STATS, COUNT, false, 4, PAIRS>(p);
}
// the deep launch of a split pass (culled scenes only); WPB = 8: the lone deep launch with the
// shading records in LDS, whose workgroups per CU the LDS bounds
template <int V, bool STATS, bool COUNT, int WPB>
__global__ __launch_bounds__(64 * WPB, (WPB == 8 && !STATS ? RT_DEEP_WIDE_WAVES : kMinWaves<V, 7, STATS>)) void render_deep_kernel(const KParams p)
{
    render_body<V, 7, STATS, COUNT, true, WPB, false>(p);
}

// ---- the reference's CUDA variant (RT_FLAG_CUDA_COMPAT) -----------------------------------
// src/CUDA/cuda_impl.cu as written, every binary32 op separately rounded in its order:
//   engine    xorshift32 per pixel, seeded with the pixel index (:16-41, :408-413); generate()
//             = float(x) * 2^-32 without a clamp (:37-41)
//   sampling  u = (float(x) + g) / W, v = (float(y) + g) / H, samples summed in order, / spp
//             (:342-351); camera without a lens offset (camera.hxx:48-50)
//   color     32 bounces by default (:63), sky mix(1, (.5,.7,1), .5 y + .5) * attenuation (:310)
//   hit       shrinking t_max, strict '<', lowest index wins ties (:131-186)
//   lambert   target = n + normalize(rius) (:197-206); metal reflect(unit d, n) +
//             normalize(rius) * roughness, absorbed unless dot > 0 (:208-222); dielectric as
//             the CPU path (:224-256), Schlick in double like raytracer.hxx:45-50
// An engine whose state is 0 stays 0 (xorshift's fixed point) and the reference's rejection
// loop would never end; here such a loop exits after one draw (only a seed that makes a
// pixel's state 0 can reach it: pixel 0 with seed 0, whose rays the default camera sends to
// the sky).
__device__ __forceinline__ float xs_gen(uint32_t &st)
{
    st ^= st << 13;
    st ^= st >> 17;
    st ^= st << 5;
    return (float)st * (1.f / 4294967296.f);
}
__device__ __forceinline__ f3 xs_unit_sphere(uint32_t &st)  // cuda_impl.cu:43-56
{
    f3 v;
    do {
        const float x = xs_gen(st) * 2.f - 1.f;
        const float y = xs_gen(st) * 2.f - 1.f;
        const float z = xs_gen(st) * 2.f - 1.f;
        v = mk(x, y, z);
    } while (v.x * v.x + v.y * v.y + v.z * v.z > 0x1.000002p+0f && st != 0u);
    return v;
}

__global__ __launch_bounds__(256) void compat_kernel(const KCompat p)
{
    const uint32_t lane = threadIdx.x & 63u;
    const float4 *shade = p.shade;
    const uint8_t *kinds = reinterpret_cast<const uint8_t *>(shade + 2 * p.n_spheres);
    const f3 org = mk(p.org[0], p.org[1], p.org[2]), llc = mk(p.llc[0], p.llc[1], p.llc[2]);
    const f3 hor = mk(p.hor[0], p.hor[1], p.hor[2]), ver = mk(p.ver[0], p.ver[1], p.ver[2]);
    const float fW = (float)p.W, fH = (float)p.H;

    uint32_t cnext = 0, cend = 0;
    bool exhausted = false, alive = false, fresh = false;
    uint32_t i = 0, x = 0, y = 0, s = 0, depth = 0, rng = 0;
    f3 o = mk(0.f, 0.f, 0.f), d = o, att = o, col = o;
    uint32_t segs = 0, tests = 0;
    for (;;) {
        // refill: idle lanes take the next pixels of the wave's chunk (64 pixels per atomic)
        uint64_t need = ballot(!alive);
        while (need && !exhausted) {
            if (cnext >= cend) {
                uint32_t c = 0;
                if (lane == 0) c = atomicAdd(p.ctr, 1u);
                c = __builtin_amdgcn_readfirstlane(c);
                if (c >= p.n_chunks) { exhausted = true; break; }
                cnext = c * 64u;
                cend = min(cnext + 64u, p.n_pixels);
            }
            const uint32_t avail = cend - cnext;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            if (!alive && rank < avail) {
                i = cnext + rank;
                const uint32_t rr = i / p.W;
                x = i - rr * p.W;
                y = p.row_offset + rr * p.row_stride;
                rng = x + y * p.W + p.seed;                 // cuda_impl.cu:408-413
                s = 0;
                col = mk(0.f, 0.f, 0.f);
                alive = fresh = true;
            }
            cnext += min((uint32_t)__popcll(need), avail);
            need = ballot(!alive);
        }
        if (ballot(alive) == 0) break;
        if (!alive) continue;
        if (fresh) {                                        // cuda_impl.cu:345-349
            const float u = ((float)x + xs_gen(rng)) / fW;
            const float v = ((float)y + xs_gen(rng)) / fH;
            o = org;
            d = (llc + hor * u) + ver * (1.f - v);
            att = mk(1.f, 1.f, 1.f);
            depth = 0;
            fresh = false;
        }
        bool done = false;
        f3 c = mk(0.f, 0.f, 0.f);
        if (depth >= p.max_depth) {
            done = true;                                    // :320
        } else {
            ++segs;
            // hit_world :171-186
            const float a = d.x * d.x + d.y * d.y + d.z * d.z;
            float tmax = RT_TMAX;
            uint32_t ib = 0xffffffffu;
            for (uint32_t k = 0; k < p.n_spheres; ++k) {
                const float4 sf = shade[2 * k];
                const float ocx = o.x - sf.x, ocy = o.y - sf.y, ocz = o.z - sf.z;
                const float b = ocx * d.x + ocy * d.y + ocz * d.z;
                const float cc = ocx * ocx + ocy * ocy + ocz * ocz - sf.w * sf.w;
                const float disc = b * b - a * cc;
                if (disc > 0.f) {
                    const float q = sqrtf(disc);
                    float t = (-b - q) / a;
                    if (!(t < tmax && t > RT_TMIN)) t = (-b + q) / a;
                    if (t < tmax && t > RT_TMIN) { tmax = t; ib = k; }
                }
            }
            tests += p.n_spheres;
            ++depth;
            if (ib == 0xffffffffu) {
                const float tt = normalize(d).y * .5f + .5f;   // :310
                c = (mk(1.f, 1.f, 1.f) * (1.f - tt) + mk(.5f, .7f, 1.f) * tt) * att;
                done = true;
            } else {
                const float4 sf = shade[2 * ib], md = shade[2 * ib + 1];
                const uint32_t kind = kinds[ib];
                const f3 hp = o + d * tmax;
                const f3 hn = (hp - mk(sf.x, sf.y, sf.z)) / sf.w;
                bool valid = true;
                f3 nd;
                if (kind == 0u) {                            // :197-206
                    nd = hn + normalize(xs_unit_sphere(rng));
                } else if (kind == 1u) {                     // :208-222
                    const f3 refl = reflect(normalize(d), hn);
                    nd = refl + normalize(xs_unit_sphere(rng)) * md.w;
                    valid = dot(nd, hn) > 0.f;
                } else {                                     // :224-256
                    const f3 ud = normalize(d);
                    f3 outward = mk(-hn.x, -hn.y, -hn.z);
                    float ri = md.w;
                    float cosv = dot(ud, hn);
                    if (cosv <= 0.f) {
                        outward = outward * -1.f;
                        ri = 1.f / ri;
                        cosv *= -1.f;
                    }
                    const f3 refr = refract(ud, outward, ri);
                    float prob = 1.f;
                    if (refr.x * refr.x + refr.y * refr.y + refr.z * refr.z > 0.f) prob = schlick(ri, cosv);
                    nd = xs_gen(rng) < prob ? reflect(ud, hn) : refr;
                }
                if (!valid) {
                    done = true;                             // :308
                } else {
                    o = hp;
                    d = nd;
                    att = att * mk(md.x, md.y, md.z);        // :303-305
                    if (depth >= p.max_depth) done = true;   // :316
                }
            }
        }
        if (done) {
            col = col + c;                                  // :350
            if (++s == p.spp) {
                col = col / (float)p.spp;                   // :353
                const uint32_t row = p.full_frame ? y : i / p.W;
                float *dst = p.out + ((size_t)row * p.W + x) * 3u;
                dst[0] = col.x;
                dst[1] = col.y;
                dst[2] = col.z;
                alive = false;
            } else {
                fresh = true;
            }
        }
    }
    if (p.segments) {
        const unsigned long long cv[2] = {segs, tests};
        for (int k = 0; k < 2; ++k) {
            unsigned long long v = cv[k];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(p.segments + k, v);
        }
    }
}

// ---- ordered accumulation of the slots, average, optional gamma/u8 --------------------
__global__ __launch_bounds__(256) void accumulate_kernel(const KAccum k)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0 && k.seg_to)
        for (int c = 0; c < 3; ++c) {
            k.seg_to[c] += k.seg_from[c];
            k.seg_from[c] = 0ull;
        }
    // the render that used this workspace has finished: reset its queue counters (no memset
    // kernel in front of the next render)
    if (k.queue_reset)
        for (uint32_t w = i; w < k.queue_words; w += gridDim.x * blockDim.x) {
            if (k.deep_over && (w & (kQueueStride - 1u)) == kDeepCount && k.queue_reset[w] > k.deep_rcap)
                *k.deep_over = k.deep_key;
            k.queue_reset[w] = 0u;
        }
    if (i >= k.n_pixels) return;
    // split passes (KAccum::part): 1 = pixels without deep samples, 2 = the others, 3 = all
    // pixels in one part; 2 and 3 clear the flags for the workspace's next pass
    // the sky kernel's pixels: their sums wait at their sample-0 slots for the
    // frame's last pass, after the sky kernel (not in part 1, which runs beside the deep launch)
    const bool sky = i >= k.sky_pos0;
    if (sky) {
        if (!k.last || k.part == 1) return;
    } else if (k.part) {
        const bool flagged = k.deep_px[i];
        if (k.part == 1 && flagged) return;
        if (k.part == 2 && !flagged) return;
        if (k.part != 1 && flagged) k.deep_px[i] = 0;
    }
    // i: the pixel's position in this pass's slots (its permuted enumeration);
    // ni: its natural enumeration index, which indexes the running sums (passes of one frame may
    // be dealt in different orders) and places the output
    const uint32_t ni = k.block_perm ? (k.block_perm[i >> 6] << 6) | (i & 63u) : i;
    f3 acc;
    if (sky) acc = mk(k.slots[3 * i], k.slots[3 * i + 1], k.slots[3 * i + 2]);
    else if (k.first) acc = mk(0.f, 0.f, 0.f);
    else acc = mk(k.acc[3 * ni], k.acc[3 * ni + 1], k.acc[3 * ni + 2]);
    // main.cxx:205 = libstdc++ reduce (<numeric>:443-460): ((c0+c1)+(c2+c3)) per block of 4,
    // blocks in order, then the spp % 4 tail one by one. Passes start on a multiple of 4.
    auto ld = [&](uint32_t s) {
        const float *v = k.slots + ((size_t)s * k.n_pixels + i) * 3u;
        return mk(v[0], v[1], v[2]);
    };
    if (sky) {
        // (summed by sky_kernel over every sample of the frame)
    } else if (k.paired) {
        // pair sums: slot 2b holds c0+c1, slot 2b+1 c2+c3 of block b; then the tail's samples
        for (uint32_t b = 0; b < k.n_blocks; ++b) acc = acc + (ld(2u * b) + ld(2u * b + 1u));
        for (uint32_t t = 4u * k.n_blocks; t < k.n_samples; ++t) acc = acc + ld(t - 2u * k.n_blocks);
    } else {
        uint32_t s = 0;
        for (; s < 4u * k.n_blocks; s += 4u) acc = acc + ((ld(s) + ld(s + 1u)) + (ld(s + 2u) + ld(s + 3u)));
        for (; s < k.n_samples; ++s) acc = acc + ld(s);
    }
    if (!k.last) {
        k.acc[3 * ni] = acc.x; k.acc[3 * ni + 1] = acc.y; k.acc[3 * ni + 2] = acc.z;
        return;
    }
    const f3 col = acc / (float)k.spp;  // main.cxx:207
    // output position
    uint32_t x, rr;
    {
        const uint32_t tiled_px = k.tiled_rows * k.W;
        if (ni < tiled_px) {
            uint32_t t = ni >> 6, w = ni & 63u;
            uint32_t ty = t / k.tiles_x, tx = t - ty * k.tiles_x;
            x = (tx << k.tile_lw) + (w & ((1u << k.tile_lw) - 1u));
            rr = (ty << (6u - k.tile_lw)) + (w >> k.tile_lw);
        } else {
            uint32_t jj = ni - tiled_px;
            rr = jj / k.W;
            x = jj - rr * k.W;
            rr += k.tiled_rows;
        }
    }
    const uint32_t row = k.full_frame ? k.row_offset + rr * k.row_stride : rr;
    const size_t o = ((size_t)row * k.W + x) * 3u;
    k.out[o] = col.x; k.out[o + 1] = col.y; k.out[o + 2] = col.z;
    if (k.out_u8) {
        // main.cxx:39-45,77-85: pow(c, 1/2.2f) then (uint8)(255 * c); powf evaluated in double
        // and rounded once (glibc's powf agrees to the last bit except at rare ties).
        const double g = (double)(1.f / 2.2f);
        k.out_u8[o] = (uint8_t)(255.f * (float)pow((double)col.x, g));
        k.out_u8[o + 1] = (uint8_t)(255.f * (float)pow((double)col.y, g));
        k.out_u8[o + 2] = (uint8_t)(255.f * (float)pow((double)col.z, g));
    }
}

// ---- the sky kernel -----------------------------------------------------
// The pixels of the tiles proven to send every primary ray to the sky: each sample is the
// reference's primary ray (main.cxx:192-200, camera.hxx:46-57) and its colour the sky's
// (main.cxx:71: background(.5 unit_direction(d).y + 1) times an attenuation of 1, exact), the
// closest hit being proven empty. One thread per pixel, its samples in order, summed in the
// blocked order of main.cxx:205's std::reduce: ((c0 + c1) + (c2 + c3)) per block of 4, added to
// the running sum block after block, then the tail samples one by one; accumulate_kernel divides
// by spp. A lane makes at most RT_SKY_CAP attempts of its lens draw per iteration and resumes
// the same sequence in the next, so the wave does not wait for its unluckiest lane's whole
// rejection run; same draws, same order, same bits. (4 threads per pixel with an LDS combine, so
// that the kernel's last waves end sooner, were not faster: profiles/r06/ab/sky_parts.txt,
// deep_sky_tail.txt; the kernel is throughput-bound on what the main launch leaves it.)
// The sky kernel's cap on lens attempts per iteration: an iteration is the sample's start, the
// attempts and its colour, so a lower cap than the main loop's (whose iterations trace a
// segment) wastes fewer attempt slots on the lanes that accepted early: per sample, iterations
// 1 / (1 - q^CAP) (q = 1 - pi/6 the rejection odds) of cost start + CAP attempts + finish
#ifndef RT_SKY_CAP
#define RT_SKY_CAP 2
#endif
__global__ __launch_bounds__(256) void sky_kernel(const KSky p)
{
    const FrameConsts &fc = p.fc;
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;  // the sky pixel
    const bool live = t < p.n_pix;
    uint32_t px, rr;
    pixel_of(fc, p.pos0 + (live ? t : 0u), px, rr, p.block_perm);
    const uint32_t py = fc.row_offset + rr * fc.row_stride;
    const uint64_t inc_data = ((uint64_t)fc.inc_data_hi << 32) | fc.inc_data_lo;
    const uint64_t inc_cam = ((uint64_t)fc.inc_cam_hi << 32) | fc.inc_cam_lo;
    const uint64_t key0 = (uint64_t)(py * fc.W + px) * fc.spp;
    const uint32_t spp = fc.spp, full_end = spp & ~3u;
    const float fW = fc.fW, fH = fc.fH, rW = fc.rW, rH = fc.rH;
    const bool dw = fc.div_fast & 1u, dh = fc.div_fast & 2u;
    const f3 org = mk(fc.org[0], fc.org[1], fc.org[2]), llc = mk(fc.llc[0], fc.llc[1], fc.llc[2]);
    const f3 hor = mk(fc.hor[0], fc.hor[1], fc.hor[2]), ver = mk(fc.ver[0], fc.ver[1], fc.ver[2]);
    // acc: the running sum; pa: the block's current pair (c0, c0 + c1, c2, c2 + c3); pb: c0 + c1
    f3 acc = mk(0.f, 0.f, 0.f), pa = acc, pb = acc;
    uint32_t s = live ? 0u : spp;
    bool started = false;
    uint64_t rc = 0;
    float uu = 0.f, vv = 0.f;
    Dbg dbg{};
    // Sample s's streams (main.cxx:192-200, key = (y W + x) spp + s): pcg_seed(key, inc) =
    // key M + inc (M + 1), and the data stream's second state M (key M + inc (M + 1)) + inc; both
    // are key M and key M^2 plus wave-uniform terms, and the key steps by 1 from sample to sample,
    // so the two products step by M and M^2 (mod 2^64, exact): no multiply per sample
    const uint64_t cd1 = inc_data * (kPcgMul + 1u), cd2 = cd1 * kPcgMul + inc_data, cc = inc_cam * (kPcgMul + 1u);
    const uint64_t mm = kPcgMul * kPcgMul;
    uint64_t km = key0 * kPcgMul, kmm = km * kPcgMul;
    const float ux = div_const((float)px, fW, rW, dw), vy = div_const((float)py, fH, rH, dh);
    while (ballot(s < spp)) {
        if (s < spp) {
            if (!started) {
                rc = km + cc;
                const float xu = fminf((float)pcg_out(km + cd1), 0x1.fffffep31f) * 0x1p-32f;  // canonical()
                const float xv = fminf((float)pcg_out(kmm + cd2), 0x1.fffffep31f) * 0x1p-32f;
                uu = ux + div_const(xu, fW, rW, dw);
                vv = vy + div_const(xv, fH, rH, dh);
                km += kPcgMul;
                kmm += mm;
                started = true;
            }
            bool got;
            const f3 r = random_in_unit_sphere_capped<false, RT_SKY_CAP>(rc, inc_cam, got, dbg);  // camera.hxx:52
            if (got) {
                const f3 rd = r * fc.lens;                                          // camera.hxx:46-57
                const f3 off = mk(uu * rd.x, vv * rd.y, 0.f);
                f3 d = ((llc + hor * uu) + ver * (1.f - vv)) - off;
                if (fc.corrected) d = d - org;
                // unit_direction(d).y (math.hxx:219-227): with |d|^2 in [2^-40, 2^40] the short
                // sqrt and division give its bits (render_body's sky)
                const float a = d.x * d.x + d.y * d.y + d.z * d.z;
                float uy;
                if (!ballot(!(a >= 0x1p-40f && a <= 0x1p40f))) {
                    const float l = sqrt_scaled(a);
                    const float y0 = __builtin_amdgcn_rcpf(l);
                    uy = div_ray(d.y, RayDiv{l, fmaf(fmaf(-l, y0, 1.f), y0, y0), 1u});
                } else {
                    uy = normalize(d).y;
                }
                const float tt = .5f * uy + 1.f;                                    // main.cxx:71
                const f3 col = mk(1.f, 1.f, 1.f) * (1.f - tt) + mk(.5f, .7f, 1.f) * tt;
                // the blocked sum as selects: pa = c0, c0 + c1, c2, c2 + c3 for s & 3 = 0..3;
                // pb keeps c0 + c1; the block's (c0 + c1) + (c2 + c3), or a tail colour, folds in
                const bool tail = s >= full_end;
                const uint32_t j = s & 3u;
                const f3 sum = pa + col;
                const bool odd = !tail && (j & 1u);
                pa = mk(odd ? sum.x : col.x, odd ? sum.y : col.y, odd ? sum.z : col.z);
                const bool first_pair = !tail && j == 1u;
                pb = mk(first_pair ? pa.x : pb.x, first_pair ? pa.y : pb.y, first_pair ? pa.z : pb.z);
                const bool fold = tail || j == 3u;
                const f3 add = pb + pa;
                const f3 fa = acc + mk(tail ? col.x : add.x, tail ? col.y : add.y, tail ? col.z : add.z);
                acc = mk(fold ? fa.x : acc.x, fold ? fa.y : acc.y, fold ? fa.z : acc.z);
                ++s;
                started = false;
            }
        }
    }
    if (live) {
        float *o = p.sums + 3u * (size_t)t;
        o[0] = acc.x;
        o[1] = acc.y;
        o[2] = acc.z;
    }
    if (p.segments) {
        const uint32_t n = lanes(live);
        if ((threadIdx.x & 63u) == 0u && n) atomicAdd(p.segments, (unsigned long long)n * spp);
    }
}

__global__ __launch_bounds__(256) void epilogue_rgb8_kernel(const float *in, uint8_t *out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double g = (double)(1.f / 2.2f);
    out[i] = (uint8_t)(255.f * (float)pow((double)in[i], g));
}

// ---- the wavefront variant (RT_FLAG_WAVEFRONT; SURVEY §8(f3), an A/B against the megakernel) ----
// Paths advance one segment per launch through ray queues in HBM: wave_gen_kernel starts one
// sample per thread (jitter, lens) and writes its ray to queue A; wave_bounce_kernel takes every
// ray of its input queue, finds the closest hit (the same culled walk and transposed member
// tests), shades it, stores finished samples to their slots and appends continuing rays to its
// output queue (one atomic per wave); the host swaps the queues max_depth times per chunk of
// items. Rejection loops run to acceptance in the thread that needs them (no deferral), so
// every stream sees the same draws in the same order as in the megakernel: same bits.
__global__ __launch_bounds__(256) void wave_gen_kernel(const KWave w)
{
    const KParams &p = w.p;
    const FrameConsts &fc = p.fc;
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    if (gid >= w.n_chunk) return;
    const uint32_t I = w.item_begin + gid;
    const uint32_t ls = udiv(I, fc.div_n_pixels);
    const uint32_t pix = I - ls * fc.n_pixels;
    uint32_t px, rr;
    pixel_of(fc, pix, px, rr, nullptr);  // (the wavefront variant deals in natural order)
    const uint32_t py = fc.row_offset + rr * fc.row_stride;
    const uint32_t sm = fc.sample_begin + ls;
    const uint64_t inc_data = ((uint64_t)fc.inc_data_hi << 32) | fc.inc_data_lo;
    const uint64_t inc_cam = ((uint64_t)fc.inc_cam_hi << 32) | fc.inc_cam_lo;
    const uint64_t km = ((uint64_t)(py * fc.W + px) * fc.spp + sm) * kPcgMul;  // pcg_seed, as render_kernel
    uint64_t rng = km + inc_data * (kPcgMul + 1u);
    uint64_t rc = km + inc_cam * (kPcgMul + 1u);
    const bool fw = fc.div_fast & 1u, fh = fc.div_fast & 2u;
    const float u = div_const((float)px, fc.fW, fc.rW, fw);
    const float v = div_const((float)py, fc.fH, fc.rH, fh);
    const float uu = u + div_const(canonical(rng, inc_data), fc.fW, fc.rW, fw);
    const float vv = v + div_const(canonical(rng, inc_data), fc.fH, fc.rH, fh);
    const f3 r = random_in_unit_sphere(rc, inc_cam);  // camera.hxx:52
    const f3 rd = r * fc.lens;                        // camera.hxx:46-57
    const f3 off = mk(uu * rd.x, vv * rd.y, 0.f);
    const f3 org = mk(fc.org[0], fc.org[1], fc.org[2]);
    const f3 o = org + off;
    f3 d = ((mk(fc.llc[0], fc.llc[1], fc.llc[2]) + mk(fc.hor[0], fc.hor[1], fc.hor[2]) * uu) +
            mk(fc.ver[0], fc.ver[1], fc.ver[2]) * (1.f - vv)) - off;
    if (fc.corrected) d = d - org;
    const RayQueue &q = w.out;
    q.f[0 * w.cap + gid] = o.x; q.f[1 * w.cap + gid] = o.y; q.f[2 * w.cap + gid] = o.z;
    q.f[3 * w.cap + gid] = d.x; q.f[4 * w.cap + gid] = d.y; q.f[5 * w.cap + gid] = d.z;
    q.f[6 * w.cap + gid] = 1.f; q.f[7 * w.cap + gid] = 1.f; q.f[8 * w.cap + gid] = 1.f;
    q.rng[gid] = rng;
    q.item[gid] = I;
    q.depth[gid] = 0u;
    if (gid == 0) *q.count = w.n_chunk;
}

template <int CULL, bool COUNT>
__global__ __launch_bounds__(256, 6) void wave_bounce_kernel(const KWave w)
{
    const KParams &p = w.p;
    extern __shared__ float4 lds_blob[];
    for (uint32_t i = threadIdx.x; i < p.lds_units; i += blockDim.x) lds_blob[i] = p.blob[i];
    __syncthreads();
    const float4 *blob = lds_blob;
    const float4 *geo = blob;
    const uint32_t *sidx = reinterpret_cast<const uint32_t *>(blob + p.n_geo);
    const float4 *clus = blob + p.clus_offset;
    __shared__ TransposeLds s_tw[4];
    TransposeLds *tw = &s_tw[threadIdx.x >> 6];
    const uint64_t inc_data = ((uint64_t)p.fc.inc_data_hi << 32) | p.fc.inc_data_lo;
    const RayQueue &qi = w.in, &qo = w.out;
    const uint32_t n = *qi.count;
    const uint32_t cap = w.cap;
    WaveTally<COUNT> wt;
    Dbg dbg{};
    // whole waves walk the queue together (the cluster walk is whole-wave code)
    for (uint32_t base = blockIdx.x * 256u; base < n; base += gridDim.x * 256u) {
        const uint32_t j = base + threadIdx.x;
        const bool live = j < n;
        const uint32_t jj = live ? j : 0u;
        f3 o = mk(qi.f[0 * cap + jj], qi.f[1 * cap + jj], qi.f[2 * cap + jj]);
        f3 d = mk(qi.f[3 * cap + jj], qi.f[4 * cap + jj], qi.f[5 * cap + jj]);
        f3 att = mk(qi.f[6 * cap + jj], qi.f[7 * cap + jj], qi.f[8 * cap + jj]);
        uint64_t rng = qi.rng[jj];
        const uint32_t I = qi.item[jj];
        uint32_t depth = qi.depth[jj];
        const bool seg = live && depth < p.max_depth;  // main.cxx:74
        const float a = d.x * d.x + d.y * d.y + d.z * d.z;
        const uint64_t segm = ballot(seg);
        const RayDiv rd = ray_div(a, segm, p.fast_roots);
        Hit h = closest_hit<false, CULL, false, COUNT>(p, geo, sidx, clus, o, d, rd, dbg, wt, seg, segm, CULL ? tw : nullptr,
                                                        no_hit());
        if (!seg) h = Hit{kNoHit};
        {
            const uint32_t ns = lanes(seg);
            wt.add_seg(ns);
            wt.add_sph((uint64_t)ns * p.n_always);
        }
        bool done = false, cont = false;
        f3 col = mk(0.f, 0.f, 0.f);
        if (live) {
            if (!seg) {
                done = true;
            } else {
                const float t = h.t();
                const uint32_t ib = h.id();
                ++depth;
                if (ib == 0xffffffffu) {  // main.cxx:71, as render_kernel
                    float uy;
                    if (rd.fd != 0u) {
                        const float l = sqrt_scaled(a);
                        const float y0 = __builtin_amdgcn_rcpf(l);
                        uy = div_ray(d.y, RayDiv{l, fmaf(fmaf(-l, y0, 1.f), y0, y0), 1u});
                    } else {
                        uy = normalize(d).y;
                    }
                    const float tt = .5f * uy + 1.f;
                    const f3 bg = mk(1.f, 1.f, 1.f) * (1.f - tt) + mk(.5f, .7f, 1.f) * tt;
                    col = bg * att;
                    done = true;
                } else if (depth >= p.max_depth) {
                    done = true;
                } else {
                    float4 sf, md;
                    uint32_t kind;
                    if (p.shade_lds) {
                        const float4 *shade = blob + p.shade_offset;
                        sf = shade[2 * ib];
                        md = shade[2 * ib + 1];
                        kind = reinterpret_cast<const uint8_t *>(shade + 2 * p.n_spheres)[ib];
                        asm volatile("");
                    } else {
                        const float4 *shade = p.blob + p.shade_offset;
                        sf = gld4(shade, 2 * ib);
                        md = gld4(shade, 2 * ib + 1);
                        kind = ((const __attribute__((address_space(1))) uint8_t *)(shade + 2 * p.n_spheres))[ib];
                    }
                    const f3 hp = o + d * t;  // math.hxx:353
                    const f3 dv = hp - mk(sf.x, sf.y, sf.z);
                    f3 hn;
                    if (p.fast_roots && all_lanes_min_abs_ok(dv)) hn = div3_short(dv, sf.w);
                    else hn = dv / sf.w;  // raytracer.hxx:71
                    att = att * mk(md.x, md.y, md.z);
                    o = hp;
                    cont = true;
                    if (kind == 0u) {  // lambert, raytracer.hxx:132-141
                        const f3 pn = hp + hn;
                        const f3 r = random_in_unit_sphere(rng, inc_data);
                        d = (pn + r) - hp;
                    } else {
                        f3 ud;
                        if (rd.fd != 0u && all_lanes_min_abs_ok(d)) ud = div3_short(d, sqrt_scaled(a));
                        else ud = normalize(d);
                        const f3 rf = reflect(ud, hn);
                        if (kind == 1u) {  // metal, :143-156
                            const f3 r = random_in_unit_sphere(rng, inc_data);
                            const f3 nd = rf + r * md.w;
                            if (dot(nd, hn) > 0.f) {
                                d = nd;
                            } else {  // absorbed: main.cxx:68, colour 0
                                cont = false;
                                done = true;
                            }
                        } else {  // dielectric, :158-194
                            const uint32_t di = p.shade_offset + 2 * p.n_spheres + (p.n_spheres + 15u) / 16u + ib;
                            float4 dcs;
                            if (p.shade_lds) {
                                dcs = blob[di];
                                asm volatile("");
                            } else {
                                dcs = gld4(p.blob, di);
                            }
                            f3 outward = mk(-hn.x, -hn.y, -hn.z);
                            float ri = md.w, xs = dcs.y;
                            float cosv = dot(ud, hn);
                            if (cosv <= 0.f) {
                                outward = outward * -1.f;
                                ri = dcs.x;
                                xs = dcs.z;
                                cosv *= -1.f;
                            }
                            const f3 refr = refract(ud, outward, ri);
                            float prob = 1.f;
                            if (refr.x * refr.x + refr.y * refr.y + refr.z * refr.z > 0.f) prob = schlick_x(xs, cosv);
                            d = canonical(rng, inc_data) < prob ? rf : refr;
                        }
                    }
                }
            }
        }
        if (done) {
            float *dst = p.slots + (size_t)I * 3u;
            dst[0] = col.x;
            dst[1] = col.y;
            dst[2] = col.z;
        }
        // continuing rays: one atomic per wave, ranks by mbcnt
        const uint64_t cm = ballot(cont);
        if (cm) {
            uint32_t b0 = 0;
            if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(cm)) b0 = atomicAdd(qo.count, (uint32_t)__popcll(cm));
            b0 = __builtin_amdgcn_readlane(b0, __builtin_ctzll(cm));
            if (cont) {
                const uint32_t k = b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
                qo.f[0 * cap + k] = o.x; qo.f[1 * cap + k] = o.y; qo.f[2 * cap + k] = o.z;
                qo.f[3 * cap + k] = d.x; qo.f[4 * cap + k] = d.y; qo.f[5 * cap + k] = d.z;
                qo.f[6 * cap + k] = att.x; qo.f[7 * cap + k] = att.y; qo.f[8 * cap + k] = att.z;
                qo.rng[k] = rng;
                qo.item[k] = I;
                qo.depth[k] = depth;
            }
        }
    }
    if (COUNT && p.segments && (threadIdx.x & 63u) == 0u) {
        atomicAdd(p.segments + 0, (unsigned long long)wt.seg);
        atomicAdd(p.segments + 1, (unsigned long long)wt.sph);
        atomicAdd(p.segments + 2, (unsigned long long)wt.box);
    }
}

// ---- launchers (called from rt_host.cpp) ---------------------------------------------
// cull: 0 = brute force (every sphere, index order), 7 = two-level cluster walk with
// transposed member tests (the default)
// COUNT: the instantiation that tallies segments and tests (when the caller passes counters)
// pairs: the pass stores sample pairs (culled scenes only)
template <int V, bool STATS, bool COUNT> static const void *ptr_cull(int cull, bool pairs)
{
    if (cull == 7) return pairs ? reinterpret_cast<const void *>(&render_kernel<V, 7, STATS, COUNT, true>)
                                : reinterpret_cast<const void *>(&render_kernel<V, 7, STATS, COUNT>);
    return pairs ? nullptr : reinterpret_cast<const void *>(&render_kernel<V, 0, STATS, COUNT>);
}

template <bool COUNT> static const void *render_ptr_c(int variant, int cull, bool pairs)
{
    switch (variant) {
    case V_EXACT_LDS: return ptr_cull<V_EXACT_LDS, false, COUNT>(cull, pairs);
    case V_FAST_LDS: return ptr_cull<V_FAST_LDS, false, COUNT>(cull, pairs);
    case V_EXACT_SCALAR:
        return cull || pairs ? nullptr : reinterpret_cast<const void *>(&render_kernel<V_EXACT_SCALAR, 0, false, COUNT>);
    case V_STATS_LDS: return ptr_cull<V_EXACT_LDS, true, true>(cull, pairs);
    default: return nullptr;
    }
}
static const void *render_ptr(int variant, int cull, bool count, bool pairs = false)
{
    return count ? render_ptr_c<true>(variant, cull, pairs) : render_ptr_c<false>(variant, cull, pairs);
}

template <bool COUNT, int WPB> static const void *render_deep_ptr_w(int variant)
{
    switch (variant) {
    case V_EXACT_LDS: return reinterpret_cast<const void *>(&render_deep_kernel<V_EXACT_LDS, false, COUNT, WPB>);
    case V_FAST_LDS: return reinterpret_cast<const void *>(&render_deep_kernel<V_FAST_LDS, false, COUNT, WPB>);
    case V_STATS_LDS: return reinterpret_cast<const void *>(&render_deep_kernel<V_EXACT_LDS, true, true, WPB>);
    default: return nullptr;
    }
}
static const void *render_deep_ptr(int variant, bool count, int wpb)
{
    if (wpb == 8) return count ? render_deep_ptr_w<true, 8>(variant) : render_deep_ptr_w<false, 8>(variant);
    if (wpb == 4) return count ? render_deep_ptr_w<true, 4>(variant) : render_deep_ptr_w<false, 4>(variant);
    return nullptr;
}

hipError_t launch_render(int variant, int cull, const KParams &p, uint32_t grid, hipStream_t stream, int wpb)
{
    // the deep launch (deep_mode != 0) exists for culled scenes only; only it has 8-wave groups
    const bool count = p.segments != nullptr;
    const void *fn = p.deep_mode ? (cull == 7 ? render_deep_ptr(variant, count, wpb) : nullptr)
                                 : (wpb == 4 ? render_ptr(variant, cull, count, p.n_pair_items != 0) : nullptr);
    if (!fn) return hipErrorInvalidValue;
    const size_t lds = (size_t)p.lds_units * 16u;
    void *args[] = {const_cast<KParams *>(&p)};
    return hipLaunchKernel(fn, dim3(grid), dim3(64u * (uint32_t)wpb), args, lds, stream);
}

// workgroups per CU and static LDS of the deep kernel with wpb waves per workgroup
hipError_t deep_occupancy(int variant, int wpb, size_t lds, int *blocks_per_cu, size_t *static_lds)
{
    const void *fn = render_deep_ptr(variant, false, wpb);
    if (!fn) return hipErrorInvalidValue;
    hipFuncAttributes a{};
    hipError_t e = hipFuncGetAttributes(&a, fn);
    if (e != hipSuccess) return e;
    *static_lds = a.sharedSizeBytes;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 64 * wpb, lds);
}

hipError_t occupancy_render(int variant, int cull, int *blocks_per_cu, size_t lds, bool pairs)
{
    const void *fn = render_ptr(variant, cull, false, pairs);
    if (!fn) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 256, lds);
}

// the static LDS of a render kernel (per-wave and per-lane arrays; the scene blob comes on top)
hipError_t static_lds_render(int variant, int cull, size_t *bytes, bool pairs)
{
    const void *fn = render_ptr(variant, cull, false, pairs);
    if (!fn) return hipErrorInvalidValue;
    hipFuncAttributes a{};
    const hipError_t e = hipFuncGetAttributes(&a, fn);
    if (e == hipSuccess) *bytes = a.sharedSizeBytes;
    return e;
}

hipError_t launch_wave_gen(const KWave &w, hipStream_t stream)
{
    hipLaunchKernelGGL(wave_gen_kernel, dim3((w.n_chunk + 255u) / 256u), dim3(256), 0, stream, w);
    return hipGetLastError();
}

static const void *wave_bounce_ptr(int cull, bool count)
{
    if (cull == 7) return count ? reinterpret_cast<const void *>(&wave_bounce_kernel<7, true>)
                                : reinterpret_cast<const void *>(&wave_bounce_kernel<7, false>);
    return count ? reinterpret_cast<const void *>(&wave_bounce_kernel<0, true>)
                 : reinterpret_cast<const void *>(&wave_bounce_kernel<0, false>);
}

hipError_t launch_wave_bounce(int cull, const KWave &w, uint32_t grid, hipStream_t stream)
{
    const size_t lds = (size_t)w.p.lds_units * 16u;
    void *args[] = {const_cast<KWave *>(&w)};
    return hipLaunchKernel(wave_bounce_ptr(cull, w.p.segments != nullptr), dim3(grid), dim3(256), args, lds, stream);
}

hipError_t occupancy_wave_bounce(int cull, int *blocks_per_cu, size_t lds)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, wave_bounce_ptr(cull, false), 256, lds);
}

hipError_t launch_compat(const KCompat &k, uint32_t grid, hipStream_t stream)
{
    hipLaunchKernelGGL(compat_kernel, dim3(grid), dim3(256), 0, stream, k);
    return hipGetLastError();
}

hipError_t occupancy_compat(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, reinterpret_cast<const void *>(&compat_kernel),
                                                        256, 0);
}

hipError_t launch_accumulate(const KAccum &k, hipStream_t stream)
{
    const uint32_t grid = (k.n_pixels + 255u) / 256u;
    hipLaunchKernelGGL(accumulate_kernel, dim3(grid), dim3(256), 0, stream, k);
    return hipGetLastError();
}

hipError_t launch_sky(const KSky &k, hipStream_t stream)
{
    if (!k.n_pix) return hipSuccess;
    hipLaunchKernelGGL(sky_kernel, dim3((k.n_pix + 255u) / 256u), dim3(256), 0, stream, k);
    return hipGetLastError();
}

hipError_t launch_epilogue(const float *in, uint8_t *out, uint64_t n, hipStream_t stream)
{
    const uint64_t grid = (n + 255u) / 256u;
    hipLaunchKernelGGL(epilogue_rgb8_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, in, out, n);
    return hipGetLastError();
}

} // namespace rt
