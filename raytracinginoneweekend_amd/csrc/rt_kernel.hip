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
__device__ __forceinline__ f3 refract(f3 I, f3 N, float eta)                          // math.hxx:300-309
{
    const float d = dot(N, I);
    const float k = 1.f - eta * eta * (1.f - d * d);
    return (I * eta - adds(N * sqrtf(k), d * eta)) * (k >= 0.f ? 1.f : 0.f);
}

// ---- RNG: PCG32 XSH-RR per (pixel, sample) stream; the increment is wave-uniform ---------
__device__ __forceinline__ uint32_t pcg_next(uint64_t &state, uint64_t inc)
{
#ifdef RT_RNG_ABLATION  // timing-only build: xorshift32 on the low word (wrong bits by design)
    uint32_t x = (uint32_t)state | 1u;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    state = (state & 0xffffffff00000000ull) | x;
    return x;
#endif
    uint64_t old = state;
    state = old * 6364136223846793005ULL + inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
}
__device__ __forceinline__ uint64_t pcg_seed(uint64_t initstate, uint64_t inc)
{
    uint64_t st = inc;  // state = 0; next() -> 0 * M + inc
    st += initstate;
    return st * 6364136223846793005ULL + inc;
}
// libstdc++ generate_canonical<float,24> over a 32-bit engine: float(x) / 2^32, kept < 1.
__device__ __forceinline__ float canonical(uint64_t &st, uint64_t inc)
{
    float r = (float)pcg_next(st, inc) * 0x1p-32f;
    return r >= 1.f ? 0x1.fffffep-1f : r;
}
// raytracer.hxx:32-43. `length(p) > 1` is evaluated as `norm(p) > 1 + 2^-23`: with a
// correctly rounded sqrt the two agree for every non-negative float (checked exhaustively,
// tests/test_numerics_cpu.py), and the loop runs as long as its slowest lane.
__device__ __forceinline__ f3 random_in_unit_sphere(uint64_t &st, uint64_t inc)
{
    f3 p;
#ifdef RT_REJECT_FIXED  // timing-only build: exactly N attempts, first accepted kept (wrong bits)
    bool got = false;
    p = mk(0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < RT_REJECT_FIXED; ++k) {
        float x = canonical(st, inc) * 2.f + -1.f;
        float y = canonical(st, inc) * 2.f + -1.f;
        float z = canonical(st, inc) * 2.f + -1.f;
        const bool ok = !got && !(x * x + y * y + z * z > 0x1.000002p+0f);
        p = ok ? mk(x, y, z) : p;
        got = got || ok;
    }
    return p;
#endif
    do {
        float x = canonical(st, inc) * 2.f + -1.f;
        float y = canonical(st, inc) * 2.f + -1.f;
        float z = canonical(st, inc) * 2.f + -1.f;
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
__device__ __forceinline__ f3 random_in_unit_sphere_capped(uint64_t &st, uint64_t inc, bool &got)
{
    if (RT_REJECT_CAP == 0) {
        got = true;
        return random_in_unit_sphere(st, inc);
    }
    f3 p = mk(0.f, 0.f, 0.f);
    got = false;
    for (int k = 0; k < (RT_REJECT_CAP > 0 ? RT_REJECT_CAP : 1); ++k) {
        const float x = canonical(st, inc) * 2.f + -1.f;
        const float y = canonical(st, inc) * 2.f + -1.f;
        const float z = canonical(st, inc) * 2.f + -1.f;
        if (!(x * x + y * y + z * z > 0x1.000002p+0f)) {
            p = mk(x, y, z);
            got = true;
            break;
        }
    }
    return p;
}

// raytracer.hxx:45-50. std::pow(float,int) promotes to double: r0 = x^2 is exact in double;
// (1-cos)^5 is formed as y^4 * y with y^4 = y^2*y^2 split exactly by an FMA, so the double
// product is within a few 1e-17 relative of glibc's pow before the final cast to float.
__device__ __forceinline__ float schlick(float ri, float c)
{
    double x = (double)((1.f - ri) / (1.f + ri));
    double r0 = x * x;
    double y = (double)(1.f - c);
    double y2 = y * y;                  // exact (24-bit * 24-bit)
    double y4 = y2 * y2;
    double y4lo = fma(y2, y2, -y4);     // exact residual
    double y5 = fma(y4, y, y4lo * y);
    return (float)(r0 + (1.0 - r0) * y5);
}

// ---- work decomposition ----------------------------------------------------------------
__device__ __forceinline__ uint32_t udiv(uint32_t n, uint32_t m, uint32_t l)
{
    if (l == 0) return n;
    const uint32_t t = __umulhi(n, m);
    return (t + ((n - t) >> 1)) >> (l - 1);
}

template <class FC>
__device__ __forceinline__ void pixel_of(const FC &fc, uint32_t i, uint32_t &x, uint32_t &rr)
{
    const uint32_t W = fc.W, tiled_rows = fc.tiled_rows, tiles_x = fc.tiles_x;
    const uint32_t tiled_px = tiled_rows * W;
    if (i < tiled_px) {
        uint32_t t = i >> 6, w = i & 63u;
        uint32_t ty = udiv(t, fc.div_tiles_x.m, fc.div_tiles_x.l), tx = t - ty * tiles_x;
        const uint32_t lw = fc.tile_lw;
        x = (tx << lw) + (w & ((1u << lw) - 1u));
        rr = (ty << (6u - lw)) + (w >> lw);
    } else {
        uint32_t j = i - tiled_px;
        rr = udiv(j, fc.div_W.m, fc.div_W.l);
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
// Diagnostic counters (STATS builds only; see rt_scene_debug_counters): per-lane tallies
// plus wave-level ones counted by the first active lane.
struct Dbg {
    uint32_t wave_blocks, lane_blocks, wave_roots, lane_roots, wave_member_blocks;
};
__device__ __forceinline__ bool first_active_lane()
{
    return (threadIdx.x & 63u) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63u);
}

struct Hit {
    float t;
    uint32_t id;   // original sphere index, 0xffffffff = none
};

template <bool FAST, bool STATS, int N = 8>
__device__ __forceinline__ void test_block8(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx, uint32_t i,
                                            f3 o, f3 d, float a, Hit &h, Dbg &dbg)
{
    float bq[N], dq[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const float4 s = geo[i + k];
        const float ocx = o.x - s.x, ocy = o.y - s.y, ocz = o.z - s.z;       // raytracer.hxx:55
        if (FAST) {  // contracted: 11 VALU per sphere
            const float b = fmaf(ocx, d.x, fmaf(ocy, d.y, ocz * d.z));
            const float c = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -s.w)));
            bq[k] = b;
            dq[k] = fmaf(b, b, -(a * c));
        } else {     // the reference's rounding, op by op: 17 VALU per sphere
            const float b = ocx * d.x + ocy * d.y + ocz * d.z;               // :57
            const float c = ocx * ocx + ocy * ocy + ocz * ocz - s.w;         // :58
            bq[k] = b;
            dq[k] = b * b - a * c;                                           // :60
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
#ifdef RT_DIVERGENT_ROOTS  // A/B build: lane-divergent branches around the root work
    if (mq[0] > 0.f) {
        if (STATS) { ++dbg.lane_blocks; if (first_active_lane()) ++dbg.wave_blocks; }
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (dq[k] > 0.f) {                                               // :62
                if (STATS) { ++dbg.lane_roots; if (first_active_lane()) ++dbg.wave_roots; }
                const float q = sqrtf(dq[k]);
                float t = (-bq[k] - q) / a;                                  // :63
                if (!(t < RT_TMAX && t > RT_TMIN)) {
                    t = (-bq[k] + q) / a;                                    // :76
                    if (!(t < RT_TMAX && t > RT_TMIN)) t = __builtin_nanf("");
                }
                const uint32_t id = sidx[i + k];
                if (t < h.t || (t == h.t && id < h.id)) { h.t = t; h.id = id; }
            }
        }
    }
#else
    // Wave-uniform branches (ballots) around the root work, lane selects inside: a masked
    // lane costs the same issue slots as a computing one, and uniform branches need no
    // exec-mask save/restore. Lanes without a positive discriminant compute throw-away
    // values (sqrt of a negative is NaN) and are excluded by `pos` in the final select.
    if (__ballot(mq[0] > 0.f)) {
        if (STATS) { ++dbg.lane_blocks; if (first_active_lane()) ++dbg.wave_blocks; }
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const bool pos = dq[k] > 0.f;                                    // :62
            if (__ballot(pos)) {
                if (STATS) { dbg.lane_roots += pos; if (first_active_lane()) ++dbg.wave_roots; }
                const float q = sqrtf(dq[k]);
                float t = (-bq[k] - q) / a;                                  // :63
                const bool ok = t < RT_TMAX && t > RT_TMIN;
                if (__ballot(pos && !ok)) {
                    const float t2 = (-bq[k] + q) / a;                       // :76
                    t = ok ? t : (t2 < RT_TMAX && t2 > RT_TMIN ? t2 : __builtin_nanf(""));
                } else {
                    t = ok ? t : __builtin_nanf("");
                }
                const uint32_t id = sidx[i + k];
                if (pos && (t < h.t || (t == h.t && id < h.id))) { h.t = t; h.id = id; }
            }
        }
    }
#endif
}

// Cluster culling: a lane tests a cluster's spheres only if its ray segment (kMIN, t_best]
// can reach the cluster's AABB grown by a pad that dominates every float error involved
// (1e-3 x (|o|_1 + max_c(|C|_1 + |e|_1)) against errors below 3e-4 of that),
// so a culled cluster never holds a sphere whose exact candidate could win: same bits.
// All boxes of a group of 32 clusters are tested first (straight-line, LDS reads batched)
// into a per-lane pass mask; the wave walks the union of the masks with a scalar loop and
// each lane runs a cluster's spheres only if its own bit is set.
#define RT_PAD_REL 1e-3f
#define RT_MAX_CLUSTERS 128  // rt_host.cpp sizes clusters so a scene never needs more

// a list of spheres: blocks of 8, then 4, then single spheres (cluster member counts are
// multiples of 4; the always-tested list has its exact count, e.g. 1 for the ground)
template <bool FAST, bool STATS>
__device__ __forceinline__ void run_members(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx,
                                            uint32_t start, uint32_t cnt, f3 o, f3 d, float a, Hit &h, Dbg &dbg)
{
    const uint32_t end = start + cnt;
    uint32_t i = start;
    for (; i + 8 <= end; i += 8) test_block8<FAST, STATS>(geo, sidx, i, o, d, a, h, dbg);
    if (i + 4 <= end) { test_block8<FAST, STATS, 4>(geo, sidx, i, o, d, a, h, dbg); i += 4; }
    for (; i < end; ++i) test_block8<FAST, STATS, 1>(geo, sidx, i, o, d, a, h, dbg);
}

struct RayBox {  // per-segment constants of the padded slab test
    float ix, iy, iz, oix, oiy, oiz, aix, aiy, aiz, px, py, pz;
};
__device__ __forceinline__ bool box_pass(const RayBox &r, float4 c0, float4 c1, float t_lo, float t_hi)
{
    const float hx = fmaf(c0.w, r.aix, r.px), hy = fmaf(c1.x, r.aiy, r.py), hz = fmaf(c1.y, r.aiz, r.pz);
    const float tcx = fmaf(c0.x, r.ix, -r.oix), tcy = fmaf(c0.y, r.iy, -r.oiy), tcz = fmaf(c0.z, r.iz, -r.oiz);
    const float tin = fmaxf(fmaxf(tcx - hx, tcy - hy), tcz - hz);
    const float tout = fminf(fminf(tcx + hx, tcy + hy), tcz + hz);
    return tin <= tout && tout >= t_lo && tin <= t_hi;
}

// Level 3: one box over every cluster (stored after the level-2 boxes). When no lane's
// segment reaches it, the wave skips the level-2 loop (returns 0 supers to walk): a ray
// that misses the padded union box misses every padded box inside it.
__device__ __forceinline__ uint32_t root_gate(const KParams &p, const RayBox &rb, const float4 *sup, float t_lo,
                                              float t_hi, uint32_t &tests)
{
    if (!p.use_root) return p.n_supers;
    ++tests;
    const bool pass = box_pass(rb, sup[2 * p.n_supers], sup[2 * p.n_supers + 1], t_lo, t_hi);
    return __ballot(pass) ? p.n_supers : 0u;
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
constexpr uint32_t kTransposeMax = 16;  // rays per transposed cluster (KParams::transpose_max <= this)
__device__ __forceinline__ uint64_t min16_u64(uint64_t k)  // minimum over each row of 16 lanes
{
    uint32_t lo = (uint32_t)k, hi = (uint32_t)(k >> 32);
    // xor 1, xor 2 (quad permutes), then half-row mirror and row mirror: every lane of a row
    // ends with the row's minimum
#define RT_MIN16_STEP(ctrl)                                                                     \
    {                                                                                           \
        const uint32_t l2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)lo, ctrl, 0xf, 0xf, false); \
        const uint32_t h2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)hi, ctrl, 0xf, 0xf, false); \
        const bool lt = h2 < hi || (h2 == hi && l2 < lo);                                       \
        lo = lt ? l2 : lo;                                                                      \
        hi = lt ? h2 : hi;                                                                      \
    }
    RT_MIN16_STEP(0xB1)
    RT_MIN16_STEP(0x4E)
    RT_MIN16_STEP(0x141)
    RT_MIN16_STEP(0x140)
#undef RT_MIN16_STEP
    return ((uint64_t)hi << 32) | lo;
}
// per-wave LDS of the transposed tests: the requesting rays by rank, and each ray's minimum
struct TransposeLds {
    float4 ray[kTransposeMax][2];   // {o.x, o.y, o.z, a}, {d.x, d.y, d.z, -}
    uint64_t key[kTransposeMax];
};
template <bool FAST>
__device__ __forceinline__ void members_transposed(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx,
                                                   uint32_t start, uint32_t cnt, uint64_t M, bool req,
                                                   TransposeLds *tw, f3 o, f3 d, float a, Hit &h)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m = (uint32_t)__popcll(M);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    if (req) {
        tw->ray[rank][0] = make_float4(o.x, o.y, o.z, a);
        tw->ray[rank][1] = make_float4(d.x, d.y, d.z, 0.f);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t k = lane & 15u;          // member slot (slots >= cnt read beyond: masked)
    const bool kval = k < cnt;
    const float4 s = geo[start + k];
    const uint32_t sid = sidx[start + k];
    for (uint32_t r0 = 0; r0 < m; r0 += 4u) {
        const uint32_t r = r0 + (lane >> 4);
        const bool valid = kval && r < m;
        const uint32_t rr = min(r, m - 1u);
        const float4 q0 = tw->ray[rr][0], q1 = tw->ray[rr][1];
        const float ra = q0.w;                                              // |d|^2, as closest_hit
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
        const bool pos = valid && disc > 0.f;                              // :62
        uint64_t key = ~0ull;
        if (__ballot(pos)) {
            const float q = sqrtf(disc);
            float t = (-b - q) / ra;                                       // :63
            const bool ok = t < RT_TMAX && t > RT_TMIN;
            if (__ballot(pos && !ok)) {
                const float t2 = (-b + q) / ra;                            // :76
                t = ok ? t : (t2 < RT_TMAX && t2 > RT_TMIN ? t2 : __builtin_nanf(""));
            } else {
                t = ok ? t : __builtin_nanf("");
            }
            if (pos && t == t) key = ((uint64_t)__float_as_uint(t) << 32) | sid;
        }
        key = min16_u64(key);
        if (k == 0u && r < m) tw->key[r] = key;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (req) {
        const uint64_t kk = tw->key[rank];
        if (kk < (((uint64_t)__float_as_uint(h.t) << 32) | h.id)) {
            h.t = __uint_as_float((uint32_t)(kk >> 32));
            h.id = (uint32_t)kk;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <bool FAST, bool STATS>
__device__ __forceinline__ void cluster_members7(bool req, uint32_t scu_lane, const float4 *__restrict__ geo,
                                                 const uint32_t *__restrict__ sidx, TransposeLds *tw, uint32_t tmax,
                                                 f3 o, f3 d, float a, Hit &h, Dbg &dbg, uint32_t &tests)
{
    const uint64_t M = __ballot(req);
    if (!M) return;
    const uint32_t scu = __builtin_amdgcn_readfirstlane(scu_lane);
    const uint32_t start = scu & 0xffffu, cnt = scu >> 16;
    if (req) tests += cnt << 16;
    if ((uint32_t)__popcll(M) <= tmax && cnt <= 16u) {
        members_transposed<FAST>(geo, sidx, start, cnt, M, req, tw, o, d, a, h);
    } else if (req) {
        if (STATS && first_active_lane()) dbg.wave_member_blocks += (cnt + 7) / 8;
        run_members<FAST, STATS>(geo, sidx, start, cnt, o, d, a, h, dbg);
    }
}

template <bool FAST, int CULL, bool STATS>
__device__ __forceinline__ Hit closest_hit(const KParams &p, const float4 *__restrict__ geo,
                                           const uint32_t *__restrict__ sidx, const float4 *__restrict__ clus, f3 o,
                                           f3 d, Dbg &dbg, uint32_t &tests, uint64_t (&cmask)[2], bool active = true,
                                           TransposeLds *tw = nullptr)
{
    const float a = d.x * d.x + d.y * d.y + d.z * d.z;
    Hit h{RT_TMAX, 0xffffffffu};
    run_members<FAST, STATS>(geo, sidx, 0, p.n_always, o, d, a, h, dbg);
#ifdef RT_DUP_ALWAYS  // timing-only build: the always-tested list twice
    {
        f3 o2 = o;
        asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
        run_members<FAST, STATS>(geo, sidx, 0, p.n_always, o2, d, a, h, dbg);
    }
#endif
    tests += p.n_always;
    if (CULL) {
        auto safe_rcp = [](float x) {
            return __builtin_amdgcn_rcpf(fabsf(x) < 1e-30f ? copysignf(1e-30f, x) : x);
        };
        const float ix = safe_rcp(d.x), iy = safe_rcp(d.y), iz = safe_rcp(d.z);
        const float oix = o.x * ix, oiy = o.y * iy, oiz = o.z * iz;
        const float aix = fabsf(ix), aiy = fabsf(iy), aiz = fabsf(iz);
        const float pad = fmaf(RT_PAD_REL, fabsf(o.x) + fabsf(o.y) + fabsf(o.z), p.clus_pad);
        const float px = pad * aix, py = pad * aiy, pz = pad * aiz;
        const float tb_hi = h.t * 1.002f;
        const float t_lo = 0.5f * RT_TMIN;
        if (CULL == 7) {
            // structure 5's walk with whole-wave control (lanes predicated by `active`), so
            // that every lane can take part in a cluster's transposed member tests
            const RayBox rb{ix, iy, iz, oix, oiy, oiz, aix, aiy, aiz, px, py, pz};
            const float4 *sup = clus + (p.supers_offset - p.clus_offset);
            uint32_t n_supers = p.n_supers;
            if (p.use_root) {
                tests += active ? 1u : 0u;
                if (!__ballot(active && box_pass(rb, sup[2 * p.n_supers], sup[2 * p.n_supers + 1], t_lo, tb_hi)))
                    n_supers = 0;
            }
            for (uint32_t g = 0; g < n_supers; ++g) {
                const float4 s0 = sup[2 * g], s1 = sup[2 * g + 1];
                tests += active ? 1u : 0u;
                bool sp = active && box_pass(rb, s0, s1, t_lo, h.t * 1.002f);
#ifdef RT_DUP_BOXES  // timing-only build: every box test twice (an opaque copy of the ray's constants)
                {
                    RayBox r2 = rb;
                    asm volatile("" : "+v"(r2.ix), "+v"(r2.iy), "+v"(r2.iz), "+v"(r2.px));
                    sp = sp && box_pass(r2, s0, s1, t_lo, h.t * 1.002f);
                }
#endif
                if (!__ballot(sp)) continue;
                const uint32_t c0i = __builtin_amdgcn_readfirstlane(__float_as_uint(s1.w)) & 0xffffu;
                tests += sp ? 4u : 0u;
                for (uint32_t c = c0i; c < c0i + 4; c += 2) {
                    const float tb_now = h.t * 1.002f;
                    const float4 a0 = clus[2 * c], a1 = clus[2 * c + 1], b0 = clus[2 * c + 2], b1 = clus[2 * c + 3];
                    bool pa = sp && box_pass(rb, a0, a1, t_lo, tb_now), pb = sp && box_pass(rb, b0, b1, t_lo, tb_now);
#ifdef RT_DUP_BOXES
                    {
                        RayBox r2 = rb;
                        asm volatile("" : "+v"(r2.ix), "+v"(r2.iy), "+v"(r2.iz), "+v"(r2.px));
                        pa = pa && box_pass(r2, a0, a1, t_lo, tb_now);
                        pb = pb && box_pass(r2, b0, b1, t_lo, tb_now);
                    }
#endif
                    cluster_members7<FAST, STATS>(pa, __float_as_uint(a1.w), geo, sidx, tw, p.transpose_max, o, d, a, h,
                                                  dbg, tests);
                    cluster_members7<FAST, STATS>(pb, __float_as_uint(b1.w), geo, sidx, tw, p.transpose_max, o, d, a, h,
                                                  dbg, tests);
                }
            }
            return h;
        }
        if (CULL == 6) {
            // boxes only: the two-level box walk of structure 5 against the always-list t_best,
            // into a per-lane mask of passing clusters; the members are tested afterwards by
            // the whole wave on compacted (ray, cluster half) units (members_compacted)
            const RayBox rb{ix, iy, iz, oix, oiy, oiz, aix, aiy, aiz, px, py, pz};
            const float4 *sup = clus + (p.supers_offset - p.clus_offset);
            const uint32_t n_supers = root_gate(p, rb, sup, t_lo, tb_hi, tests);
            for (uint32_t g = 0; g < n_supers; ++g) {
                const float4 s0 = sup[2 * g], s1 = sup[2 * g + 1];
                ++tests;
                if (!box_pass(rb, s0, s1, t_lo, tb_hi)) continue;
                const uint32_t c0i = __builtin_amdgcn_readfirstlane(__float_as_uint(s1.w)) & 0xffffu;
                tests += 4;
                uint32_t bits = 0;
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k)
                    bits |= box_pass(rb, clus[2 * (c0i + k)], clus[2 * (c0i + k) + 1], t_lo, tb_hi) ? (1u << k) : 0u;
                const uint64_t sh = (uint64_t)bits << (c0i & 63u);
                if (c0i < 64u) cmask[0] |= sh;
                else cmask[1] |= sh;
            }
            return h;
        }
        if (CULL == 5) {
            // two levels: a box over each 4 clusters, then pairs of cluster boxes inside
            const RayBox rb{ix, iy, iz, oix, oiy, oiz, aix, aiy, aiz, px, py, pz};
            const float4 *sup = clus + (p.supers_offset - p.clus_offset);
            const uint32_t n_supers = root_gate(p, rb, sup, t_lo, tb_hi, tests);
            for (uint32_t g = 0; g < n_supers; ++g) {
                const float4 s0 = sup[2 * g], s1 = sup[2 * g + 1];
                ++tests;
                if (!box_pass(rb, s0, s1, t_lo, h.t * 1.002f)) continue;
                const uint32_t c0i = __builtin_amdgcn_readfirstlane(__float_as_uint(s1.w)) & 0xffffu;
                tests += 4;
                for (uint32_t c = c0i; c < c0i + 4; c += 2) {
                    const float tb_now = h.t * 1.002f;
                    const float4 a0 = clus[2 * c], a1 = clus[2 * c + 1], b0 = clus[2 * c + 2], b1 = clus[2 * c + 3];
                    const bool pa = box_pass(rb, a0, a1, t_lo, tb_now), pb = box_pass(rb, b0, b1, t_lo, tb_now);
                    if (pa) {
                        const uint32_t scu = __builtin_amdgcn_readfirstlane(__float_as_uint(a1.w));
                        const uint32_t start = scu & 0xffffu, cnt = scu >> 16;
                        if (STATS && first_active_lane()) dbg.wave_member_blocks += (cnt + 7) / 8;
                        run_members<FAST, STATS>(geo, sidx, start, cnt, o, d, a, h, dbg);
#ifdef RT_DUP_MEMBERS  // timing-only build: each passing cluster's members twice
                        {
                            f3 o2 = o;
                            asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
                            run_members<FAST, STATS>(geo, sidx, start, cnt, o2, d, a, h, dbg);
                        }
#endif
                        tests += cnt << 16;
                    }
                    if (pb) {
                        const uint32_t scu = __builtin_amdgcn_readfirstlane(__float_as_uint(b1.w));
                        const uint32_t start = scu & 0xffffu, cnt = scu >> 16;
                        if (STATS && first_active_lane()) dbg.wave_member_blocks += (cnt + 7) / 8;
                        run_members<FAST, STATS>(geo, sidx, start, cnt, o, d, a, h, dbg);
#ifdef RT_DUP_MEMBERS  // timing-only build: each passing cluster's members twice
                        {
                            f3 o2 = o;
                            asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
                            run_members<FAST, STATS>(geo, sidx, start, cnt, o2, d, a, h, dbg);
                        }
#endif
                        tests += cnt << 16;
                    }
                }
            }
            return h;
        }
        if (CULL == 1 || (CULL >= 3 && CULL <= 4)) {
            // interleaved: boxes of G clusters (G = 1, or 2/4 with their LDS reads issued
            // together), then each passing cluster's spheres. The box tests of a group use the
            // t_best from before the group: older, larger, still conservative.
            constexpr uint32_t G = CULL == 1 ? 1u : (CULL == 3 ? 2u : 4u);
            for (uint32_t c = 0; c < p.n_clusters; c += G) {
                bool pass[G];
                uint32_t sc[G];
                const float tb_now = h.t * 1.002f;
#pragma unroll
                for (uint32_t g = 0; g < G; ++g) {
                    const float4 c0 = clus[2 * (c + g)], c1 = clus[2 * (c + g) + 1];
                    const float hx = fmaf(c0.w, aix, px), hy = fmaf(c1.x, aiy, py), hz = fmaf(c1.y, aiz, pz);
                    const float tcx = fmaf(c0.x, ix, -oix), tcy = fmaf(c0.y, iy, -oiy), tcz = fmaf(c0.z, iz, -oiz);
                    const float tin = fmaxf(fmaxf(tcx - hx, tcy - hy), tcz - hz);
                    const float tout = fminf(fminf(tcx + hx, tcy + hy), tcz + hz);
                    pass[g] = tin <= tout && tout >= t_lo && tin <= tb_now;
                    sc[g] = __float_as_uint(c1.w);
                }
#pragma unroll
                for (uint32_t g = 0; g < G; ++g) {
                    if (pass[g]) {
                        const uint32_t scu = __builtin_amdgcn_readfirstlane(sc[g]);
                        const uint32_t start = scu & 0xffffu, cnt = scu >> 16;
                        if (STATS && first_active_lane()) dbg.wave_member_blocks += (cnt + 7) / 8;
                        run_members<FAST, STATS>(geo, sidx, start, cnt, o, d, a, h, dbg);
                        tests += cnt << 16;
                    }
                }
            }
            tests += p.n_clusters_real;
            return h;
        }
        // pass 1: every box (<= RT_MAX_CLUSTERS), masks per group of 32
        uint32_t masks[RT_MAX_CLUSTERS / 32], unions[RT_MAX_CLUSTERS / 32];
#pragma unroll
        for (uint32_t gi = 0; gi < RT_MAX_CLUSTERS / 32; ++gi) {
            const uint32_t g = gi * 32;
            uint32_t mask = 0, any = 0;  // any: wave union, from ballots (active lanes only)
            if (g < p.n_clusters) {
                const uint32_t ng = min(32u, p.n_clusters - g);

#pragma unroll 1
                for (uint32_t c = 0; c < ng; ++c) {
                    const float4 c0 = clus[2 * (g + c)], c1 = clus[2 * (g + c) + 1];  // {C, ex}, {ey, ez, -, start|count}
                    const float hx = fmaf(c0.w, aix, px), hy = fmaf(c1.x, aiy, py), hz = fmaf(c1.y, aiz, pz);
                    const float tcx = fmaf(c0.x, ix, -oix), tcy = fmaf(c0.y, iy, -oiy), tcz = fmaf(c0.z, iz, -oiz);
                    const float tin = fmaxf(fmaxf(tcx - hx, tcy - hy), tcz - hz);
                    const float tout = fminf(fminf(tcx + hx, tcy + hy), tcz + hz);
                    const bool pass = tin <= tout && tout >= t_lo && tin <= tb_hi;
                    mask |= pass ? (1u << c) : 0u;
                    any |= __ballot(pass) ? (1u << c) : 0u;
                }
            }
            masks[gi] = mask;
            unions[gi] = any;
        }
        tests += p.n_clusters_real;
        // pass 2: the wave walks the union of the lanes' masks
#pragma unroll
        for (uint32_t gi = 0; gi < RT_MAX_CLUSTERS / 32; ++gi) {
            const uint32_t g = gi * 32;
            if (g >= p.n_clusters) break;
            const uint32_t mask = masks[gi];
            uint32_t u = __builtin_amdgcn_readfirstlane(unions[gi]);
            while (u) {
                const uint32_t c = __builtin_ctz(u);
                u &= u - 1u;
                if (mask & (1u << c)) {
                    const uint32_t sc = __float_as_uint(clus[2 * (g + c) + 1].w);
                    const uint32_t start = __builtin_amdgcn_readfirstlane(sc & 0xffffu);
                    const uint32_t cnt = __builtin_amdgcn_readfirstlane(sc >> 16);
                    run_members<FAST, STATS>(geo, sidx, start, cnt, o, d, a, h, dbg);
                    tests += cnt << 16;
                }
            }
        }
    }
    return h;
}

// Structure 6, phase B: the member tests of every (lane, passing cluster) pair of the wave,
// compacted. A pair is split into units of 8 member slots (cluster_units per cluster); the
// units are numbered by an exclusive prefix over the lanes (bit-plane ballots), dealt 64 per
// round to ALL lanes of the wave (idle lanes included), and each unit's best candidate is
// folded into its owner's LDS key with one ds_min_u64: key = bits(t) << 32 | original index,
// and for t > 0 the u64 order IS the (t, index) lexicographic order of closest_hit, so the
// result is the same whatever lane tests what, in whatever order. A half-block reading past
// its cluster tests the next cluster's spheres (or never-hitting padding): extra genuine
// candidates never change the minimum. Must be called by the whole wave (uniform control).
template <bool FAST, bool STATS>
__device__ __forceinline__ void members_compacted(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx,
                                                  const float4 *__restrict__ clus, uint64_t *wkey, uint32_t *wlist,
                                                  const uint64_t (&cmask)[2], f3 o, f3 d, Hit &h, Dbg &dbg,
                                                  uint32_t &tests, uint32_t p_units)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t k = (uint32_t)(__popcll(cmask[0]) + __popcll(cmask[1]));  // passing clusters
    // exclusive prefix E of k over the lanes, and the wave total T
    uint32_t E = 0, T = 0;
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
        const uint64_t bb = __ballot((k >> b) & 1u);
        E += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
        T += (uint32_t)__popcll(bb) << b;
    }
    T = __builtin_amdgcn_readfirstlane(T);
    if (T == 0) return;
    if (k) wkey[lane] = ((uint64_t)__float_as_uint(h.t) << 32) | h.id;
    const uint32_t U = p_units;  // blocks of 8 per cluster (cluster size / 8, rounded up)
    const uint32_t units = U * T;
    for (uint32_t base = 0; base < units; base += 64u) {
        // emission: each owner writes its units in [base, base + 64)
        if (k) {
            uint32_t j = 0;
#pragma unroll
            for (int w = 0; w < 2; ++w) {
                uint64_t m = cmask[w];
                while (m) {
                    const uint32_t c = (uint32_t)__builtin_ctzll(m) + 64u * (uint32_t)w;
                    m &= m - 1u;
                    const uint32_t u0 = U * (E + j++);
                    if (u0 + U > base && u0 < base + 64u) {
                        const uint32_t e = lane | (c << 6);
                        for (uint32_t hb = 0; hb < U; ++hb)
                            if (u0 + hb >= base && u0 + hb < base + 64u) wlist[u0 + hb - base] = e | (hb << 13);
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t n_here = min(64u, units - base);
        const uint32_t e = lane < n_here ? wlist[lane] : 0u;
        const uint32_t owner = e & 63u;
        // the owner's ray, read across lanes (every lane active here)
        const f3 ro = mk(__shfl(o.x, owner), __shfl(o.y, owner), __shfl(o.z, owner));
        const f3 rd = mk(__shfl(d.x, owner), __shfl(d.y, owner), __shfl(d.z, owner));
        if (lane < n_here) {
            const uint32_t c = (e >> 6) & 127u, half = e >> 13;  // half: the unit's block of 8
            const uint32_t sc = __float_as_uint(clus[2 * c + 1].w);
            const uint32_t start = sc & 0xffffu, cnt = sc >> 16;
            if (8u * half < cnt) {
                const float a = rd.x * rd.x + rd.y * rd.y + rd.z * rd.z;
                Hit u{RT_TMAX, 0xffffffffu};
                test_block8<FAST, STATS>(geo, sidx, start + 8u * half, ro, rd, a, u, dbg);
                tests += 8u << 16;
                if (u.id != 0xffffffffu)
                    atomicMin((unsigned long long *)(wkey + owner), ((uint64_t)__float_as_uint(u.t) << 32) | u.id);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (k) {
        const uint64_t key = wkey[lane];
        h.t = __uint_as_float((uint32_t)(key >> 32));
        h.id = (uint32_t)key;
    }
}

// ---- the megakernel ----------------------------------------------------------------------
#ifndef RT_MIN_WAVES_PER_SIMD
#define RT_MIN_WAVES_PER_SIMD 1  // measured: forcing 8 waves (64 VGPRs) spills and runs slower
#endif
// ---- deep paths: one wave per workgroup takes them over --------------------------------
// 0.18% of config 3's samples never leave the glass sphere and run to max_depth; those and
// other deep paths are 10% of the segments but, spread over every wave, make almost every
// wave iteration pay for their dielectric shading and cluster members. With DEEP, waves 0-2 of
// a workgroup park a path that is about to trace segment p.deep_depth + 1 in a workgroup LDS
// queue (when it has room) and refill the lane; wave 3 takes parked paths before new items,
// so deep paths share waves with each other. The result is unchanged: a path's state moves
// whole, and every sample still lands in its own slot.
constexpr uint32_t kDeepQ = 64;
struct DeepQueue {
    uint32_t head, tail, producers, pad;  // head: claimed by producers; tail: consumed by wave 3
    uint32_t gen[kDeepQ];                 // slot generation (pos / kDeepQ + 1) once written
    uint4 st[kDeepQ][5];                  // bits of o, d, att, {rng lo, rng hi, pix, ls}, pn
    uint32_t meta[kDeepQ];                // depth | pend << 8 | pend_metal << 9
};

// Structure 7 (the default) is held to 6 waves per SIMD: unhinted it takes 83 VGPRs (5 waves);
// hinted, the allocator keeps 79 and parks one 12-byte constant that only the metal-absorption
// path reloads (measured: 5.03-5.06 ms vs 5.19-5.24 per config-3 launch).
template <int V, int CULL, bool STATS, bool DEEP>
constexpr int kMinWaves = (CULL == 7 && !STATS && !DEEP) ? 6 : RT_MIN_WAVES_PER_SIMD;
template <int V, int CULL, bool STATS, bool DEEP>
__global__ __launch_bounds__(256, (kMinWaves<V, CULL, STATS, DEEP>)) void render_kernel(const KParams p)
{
    constexpr bool FAST = (V == V_FAST_LDS);
    // Scene blob -> LDS (or read in place from global for the scalar-cache A/B variant):
    // [geo float4 x n_geo][sidx u32 x n_geo, 16-B padded][clusters float4 x 2 x n_clusters]
    extern __shared__ float4 lds_blob[];
    const float4 *blob;
    DeepQueue *dq = nullptr;
    if constexpr (DEEP) {
        __shared__ DeepQueue s_dq;
        dq = &s_dq;
        if (threadIdx.x < kDeepQ) dq->gen[threadIdx.x] = 0u;
        if (threadIdx.x == 0) { dq->head = 0u; dq->tail = 0u; dq->producers = 3u; }
    }
    if constexpr (V == V_EXACT_SCALAR) {
        blob = p.blob;
        if (DEEP) __syncthreads();
    } else {
        for (uint32_t i = threadIdx.x; i < p.lds_units; i += blockDim.x) lds_blob[i] = p.blob[i];
        __syncthreads();
        blob = lds_blob;
    }
    const bool deep_wave = DEEP && (threadIdx.x >> 6) == 3u;  // the consumer of parked paths
    uint32_t qtail = 0;                                        // deep wave: its copy of dq->tail
    // Per-render constants used only where a sample or an item starts are re-read from the
    // kernarg segment at each use (scalar loads) through a pointer made opaque every loop
    // iteration, so they do not pin ~30 SGPRs for the whole kernel (SGPR count bounds the
    // workgroups per CU on gfx950).
    typedef const __attribute__((address_space(4))) FrameConsts *fc_ptr_t;
    const fc_ptr_t fc_base =
        (fc_ptr_t)((const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr() +
                   offsetof(KParams, fc));
    const float4 *geo = blob;
    const uint32_t *sidx = reinterpret_cast<const uint32_t *>(blob + p.n_geo);
    const float4 *clus = blob + p.clus_offset;

    const uint32_t lane = threadIdx.x & 63u;
    // structure 6: per-wave LDS scratch of the compacted member tests (owner keys, unit list)
    uint64_t *wkey = nullptr;
    uint32_t *wlist = nullptr;
    TransposeLds *tw = nullptr;
    if constexpr (CULL == 7) {
        __shared__ TransposeLds s_tw[4];
        tw = &s_tw[threadIdx.x >> 6];
    }
    if constexpr (CULL == 6) {
        __shared__ uint64_t s_wkey[4][64];
        __shared__ uint32_t s_wlist[4][64];
        wkey = s_wkey[threadIdx.x >> 6];
        wlist = s_wlist[threadIdx.x >> 6];
    }

    // wave-uniform cursor over the item space
    uint32_t q = blockIdx.x & 7u, q_tried = 0;
    uint32_t cnext = 0, cend = 0;
    bool exhausted = false;

    // lane state: the lane's item is one sample (pixel enumeration index, sample of the pass)
    bool alive = false;
    uint32_t pix = 0, ls = 0;
    f3 o = mk(0.f, 0.f, 0.f), d = o, att = o;
    uint32_t depth = 0;
    uint64_t rng = 0;
    // a lambert/metal hit leaves its scatter offset to the next iteration's rejection loop:
    // o = hit point; d = p + n (lambert) or reflect(unit(d), n) (metal); pn = n, roughness
    bool pend = false, pend_metal = false;
    // a fresh sample whose lens draw did not finish within RT_REJECT_CAP attempts: its camera
    // stream state waits in (o.x, o.y) and its jittered (u, v) in (d.x, d.y) until it does
    bool pend_lens = false;
    float4 pn = make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t segs = 0, tests_sph = 0, tests_box = 0;  // per-lane tallies (widened at the end)
    Dbg dbg{0, 0, 0, 0, 0};
    uint32_t dbg_iters = 0, dbg_refills = 0, dbg_iters_dry = 0;
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
        fc_ptr_t fc = fc_base;
        asm volatile("" : "+s"(fc));
        // ---- refill items for idle lanes and start their samples -------------------
        uint64_t need = __ballot(!alive);
        bool fresh = false;
        if (DEEP && deep_wave && need) {
            // parked paths first, in queue order; a slot is read once its producer has
            // published it (generation), and tail moves only after the reads
            const uint32_t h = __builtin_amdgcn_readfirstlane(__atomic_load_n(&dq->head, __ATOMIC_ACQUIRE));
            const uint32_t k = min((uint32_t)__popcll(need), h - qtail);
            if (k) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                if (!alive && rank < k) {
                    const uint32_t pos = qtail + rank, sl = pos % kDeepQ;
                    while (__atomic_load_n(&dq->gen[sl], __ATOMIC_ACQUIRE) != pos / kDeepQ + 1u)
                        __builtin_amdgcn_s_sleep(1);
                    const uint4 a0 = dq->st[sl][0], a1 = dq->st[sl][1], a2 = dq->st[sl][2], a3 = dq->st[sl][3];
                    const uint4 a4 = dq->st[sl][4];
                    const uint32_t mt = dq->meta[sl];
                    o = mk(__uint_as_float(a0.x), __uint_as_float(a0.y), __uint_as_float(a0.z));
                    d = mk(__uint_as_float(a1.x), __uint_as_float(a1.y), __uint_as_float(a1.z));
                    att = mk(__uint_as_float(a2.x), __uint_as_float(a2.y), __uint_as_float(a2.z));
                    pn = make_float4(__uint_as_float(a4.x), __uint_as_float(a4.y), __uint_as_float(a4.z),
                                     __uint_as_float(a4.w));
                    rng = ((uint64_t)a3.y << 32) | a3.x;
                    pix = a3.z;
                    ls = a3.w;
                    depth = mt & 0xffu;
                    pend = (mt >> 8) & 1u;
                    pend_metal = (mt >> 9) & 1u;
                    alive = true;
                }
                qtail += k;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __atomic_store_n(&dq->tail, qtail, __ATOMIC_RELEASE);
                need = __ballot(!alive);
            }
        }
        if (STATS && need && !exhausted && lane == 0) ++dbg_refills;
        while (need && !exhausted) {
            if (cnext >= cend) {
                uint32_t c = 0;
                if (lane == 0) c = atomicAdd(p.queue_ctr + q * kQueueStride, 1u);
                c = __builtin_amdgcn_readfirstlane(c);
                if (p.guided_l2b < 0.f) {
                    // guided: queue q owns blocks [qb0, qb1) of 64 items; ticket c takes blocks
                    // [S(c), S(c+1)), S(t) = min(B, floor(B (1 - beta^t)) + 2t): chunks shrink
                    // geometrically from ~B / (K waves per queue) to 2 blocks, so a queue is
                    // served by few atomics and its last chunks are small. S is the same
                    // function for every wave, so consecutive tickets tile the range; the 2t
                    // term keeps it increasing even if exp2 or the float product is off by an
                    // ulp (one block at most).
                    const uint32_t qb0 = (uint32_t)(((uint64_t)p.n_blocks * q) >> 3);
                    const uint32_t B = (uint32_t)(((uint64_t)p.n_blocks * (q + 1u)) >> 3) - qb0;
                    auto S = [&](uint32_t t) -> uint32_t {
                        const float x = t ? exp2f((float)t * p.guided_l2b) : 1.f;
                        const uint64_t g = (uint64_t)floorf((float)B * (1.f - x)) + 2ull * t;
                        return g < B ? (uint32_t)g : B;
                    };
                    const uint32_t s0 = S(c);
                    if (s0 >= B) {
                        q = (q + 1u) & 7u;
                        if (++q_tried == 8u) exhausted = true;
                        continue;
                    }
                    cnext = 64u * (qb0 + s0);
                    cend = min(64u * (qb0 + S(c + 1u)), p.n_items);
                } else {
                const uint64_t chunk = (uint64_t)q + 8ull * c;
                if (chunk >= p.n_chunks) {
                    q = (q + 1u) & 7u;
                    if (++q_tried == 8u) exhausted = true;
                    continue;
                }
                // big chunks first, then 64-item chunks for the end of the launch: a wave
                // then holds at most 64 undealt items when the queues run dry
                if (chunk < p.n_big_chunks) {
                    cnext = (uint32_t)chunk * p.chunk_items;
                    cend = cnext + p.chunk_items;
                } else {
                    cnext = p.n_big_chunks * p.chunk_items + ((uint32_t)chunk - p.n_big_chunks) * 64u;
                    cend = min(cnext + 64u, p.n_items);
                }
                }
            }
            const uint32_t avail = cend - cnext;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            if (!alive && rank < avail) {
                const uint32_t I = cnext + rank;
                ls = udiv(I, fc->div_n_pixels.m, fc->div_n_pixels.l);
                pix = I - ls * fc->n_pixels;
                alive = fresh = true;
            }
            const uint32_t took = min((uint32_t)__popcll(need), avail);
            cnext += took;
            need = __ballot(!alive);
        }

        stamp(0);
        // ---- start the sample of a freshly assigned item (main.cxx:192-200) -----------
        const uint64_t inc_data = ((uint64_t)fc->inc_data_hi << 32) | fc->inc_data_lo;
        uint64_t rc = 0;  // the camera stream of a fresh sample
        float uu = 0.f, vv = 0.f;
        if (fresh) {
            uint32_t px, rr;
            pixel_of(*fc, pix, px, rr);
            const uint32_t py = fc->row_offset + rr * fc->row_stride;
            const uint32_t s = fc->sample_begin + ls;
            const uint64_t key = ((uint64_t)py * fc->W + px) * fc->spp + s;
            const uint64_t inc_cam = ((uint64_t)fc->inc_cam_hi << 32) | fc->inc_cam_lo;
            rng = pcg_seed(key, inc_data);
            rc = pcg_seed(key, inc_cam);
            const float fW = fc->fW, fH = fc->fH;
            const float u = (float)px / fW;
            const float v = (float)py / fH;
            uu = u + canonical(rng, inc_data) / fW;
            vv = v + canonical(rng, inc_data) / fH;
            att = mk(1.f, 1.f, 1.f);
            depth = 0;
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
        const bool lens = fresh || pend_lens;
        if (lens || pend) {
            const uint64_t inc = lens ? (((uint64_t)fc->inc_cam_hi << 32) | fc->inc_cam_lo) : inc_data;
            if (pend_lens) {
                uu = d.x;
                vv = d.y;
                rc = ((uint64_t)__float_as_uint(o.y) << 32) | __float_as_uint(o.x);
            }
            uint64_t st = lens ? rc : rng;
#ifdef RT_DUP_REJECT  // timing-only build: the rejection loop twice (the copy is discarded)
            {
                uint64_t st2 = st;
                asm volatile("" : "+v"(st2));
                const f3 r2 = random_in_unit_sphere(st2, inc);
                float sink = r2.x + r2.y + r2.z;
                asm volatile("" ::"v"(sink));
            }
#endif
            bool got;
            const f3 r = random_in_unit_sphere_capped(st, inc, got);
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
                rng = st;
                if (!pend_metal) {
                    d = (d + r) - o;                       // lambert :135, d held p + n, o = p
                } else {
                    const f3 nd = d + r * pn.w;            // metal :147, d held reflect(unit(d), n)
                    if (dot(nd, mk(pn.x, pn.y, pn.z)) > 0.f) {
                        d = nd;
                    } else {                               // absorbed: main.cxx:68, colour 0
                        alive = false;
                        float *dst = p.slots + ((size_t)ls * fc->n_pixels + pix) * 3u;
                        dst[0] = 0.f;
                        dst[1] = 0.f;
                        dst[2] = 0.f;
                    }
                }
                pend = false;
            }
        }
        stamp(1);
        if (__ballot(alive) == 0) {  // only when the item space is exhausted
            if (!DEEP || !deep_wave) break;
            // the deep wave leaves once no producer is left and the queue is empty
            const uint32_t h = __builtin_amdgcn_readfirstlane(__atomic_load_n(&dq->head, __ATOMIC_ACQUIRE));
            const uint32_t pr = __builtin_amdgcn_readfirstlane(__atomic_load_n(&dq->producers, __ATOMIC_ACQUIRE));
            if (pr == 0u && h == qtail) break;
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        if (STATS && lane == 0) {
            ++dbg_iters;
            if (exhausted) {
                if (!dbg_iters_dry) t_dry = __builtin_amdgcn_s_memrealtime();
                ++dbg_iters_dry;
            }
        }

        // ---- closest hit of one segment for every live lane -----------------------------
        const bool seg = alive && !defer && depth < p.max_depth;  // depth check: main.cxx:74
        Hit h{RT_TMAX, 0xffffffffu};
        uint64_t cmask[2] = {0, 0};
        uint32_t tally = 0;  // low 16 bits: always-list spheres + box tests; high: member spheres
        if constexpr (CULL == 7) {  // whole wave: every lane helps with transposed member tests
            h = closest_hit<FAST, CULL, STATS>(p, geo, sidx, clus, o, d, dbg, tally, cmask, seg, tw);
            if (!seg) {
                h = Hit{RT_TMAX, 0xffffffffu};
                tally = 0;
            }
        } else if (seg) {
            h = closest_hit<FAST, CULL, STATS>(p, geo, sidx, clus, o, d, dbg, tally, cmask);
        }
#ifdef RT_DUP_HIT  // timing-only build: the closest-hit search twice on an opaque copy of the ray
        if (seg) {
            f3 o2 = o;
            asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
            uint32_t t2 = 0;
            uint64_t cm2[2] = {0, 0};
            const Hit h2 = closest_hit<FAST, CULL, STATS>(p, geo, sidx, clus, o2, d, dbg, t2, cm2);
            if (h2.t < h.t) h = h2;
        }
#endif
        if constexpr (CULL == 6)
            members_compacted<FAST, STATS>(geo, sidx, clus, wkey, wlist, cmask, o, d, h, dbg, tally, p.cluster_units);
        stamp(2);
        {
            const uint32_t al = seg ? p.n_always : 0u;
            tests_sph += al + (tally >> 16);
            tests_box += (tally & 0xffffu) - al;
        }

        // ---- shading: the hit of every live lane -----------------------------------------
        if (alive && !defer) {
            bool done = false;
            f3 col = mk(0.f, 0.f, 0.f);
            if (!seg) {
                done = true;  // main.cxx:74 (only reachable with max_depth == 0)
            } else {
                ++segs;
                const float t = h.t;
                const uint32_t ib = h.id;
                ++depth;
                if (ib == 0xffffffffu) {
                    // main.cxx:71: background(.5 * unit_direction.y + 1) * attenuation
                    const float tt = .5f * normalize(d).y + 1.f;
                    const f3 bg = mk(1.f, 1.f, 1.f) * (1.f - tt) + mk(.5f, .7f, 1.f) * tt;
                    col = bg * att;
                    done = true;
                } else if (depth >= p.max_depth) {
                    // main.cxx:65-74: a scattered ray would not be traced and an absorbed one
                    // returns 0 too; this sample's streams are not drawn from again
                    done = true;
                } else {
                    float4 sf, md;
                    uint32_t kind;
                    if (V != V_EXACT_SCALAR && p.shade_lds) {
                        const float4 *shade = blob + p.shade_offset;
                        sf = shade[2 * ib];
                        md = shade[2 * ib + 1];
                        kind = reinterpret_cast<const uint8_t *>(shade + 2 * p.n_spheres)[ib];
                    } else {
                        const float4 *shade = p.blob + p.shade_offset;
                        sf = shade[2 * ib];
                        md = shade[2 * ib + 1];
                        kind = reinterpret_cast<const uint8_t *>(shade + 2 * p.n_spheres)[ib];
                    }
                    const f3 ctr = mk(sf.x, sf.y, sf.z);
                    const f3 hp = o + d * t;                    // ray::point_at, math.hxx:353
                    const f3 hn = (hp - ctr) / sf.w;            // raytracer.hxx:71
                    att = att * mk(md.x, md.y, md.z);           // main.cxx:65 (unused if absorbed)
                    // raytracer.hxx:120-199
                    o = hp;
                    if (kind == 0u) {                           // lambert, :132-141
                        d = hp + hn;                            // + rius next iteration, then - p
                        pend = true;
                        pend_metal = false;
                    } else {
                        // metal and dielectric lanes share one unit direction and one reflection
                        // (one code path for the wave instead of two)
                        const f3 ud = normalize(d);
                        const f3 rf = reflect(ud, hn);
                        if (kind == 1u) {                       // metal, :143-156
                            d = rf;                             // + rius * roughness next iteration
                            pn = make_float4(hn.x, hn.y, hn.z, md.w);
                            pend = true;
                            pend_metal = true;
                        } else {                                // dielectric, :158-194
#ifdef RT_DUP_DIEL  // timing-only build: the dielectric shading twice on an opaque copy (result discarded)
                            {
                                f3 u2 = ud;
                                asm volatile("" : "+v"(u2.x), "+v"(u2.y), "+v"(u2.z));
                                f3 ow2 = mk(-hn.x, -hn.y, -hn.z);
                                float ri2 = md.w, c2 = dot(u2, hn);
                                if (c2 <= 0.f) { ow2 = ow2 * -1.f; ri2 = 1.f / ri2; c2 *= -1.f; }
                                const f3 rr2 = refract(u2, ow2, ri2);
                                float pr2 = 1.f;
                                if (rr2.x * rr2.x + rr2.y * rr2.y + rr2.z * rr2.z > 0.f) pr2 = schlick(ri2, c2);
                                uint64_t st2 = rng;
                                asm volatile("" : "+v"(st2));
                                const float sink = canonical(st2, inc_data) < pr2 ? rr2.x : rr2.y;
                                asm volatile("" ::"v"(sink));
                            }
#endif
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
                            // length(refr) > 0 <=> norm > 0 (correctly rounded sqrt; NaN -> false)
                            if (refr.x * refr.x + refr.y * refr.y + refr.z * refr.z > 0.f) prob = schlick(ri, cosv);
                            d = canonical(rng, inc_data) < prob ? rf : refr;
                        }
                    }
                }
            }
            stamp(3);
            if (done) {
                // the sample's colour goes to its slot; accumulate_kernel forms the reference's
                // blocked sum over the slots (main.cxx:205)
                alive = false;
                float *dst = p.slots + ((size_t)ls * fc->n_pixels + pix) * 3u;
                dst[0] = col.x;
                dst[1] = col.y;
                dst[2] = col.z;
            }
        }
        if constexpr (DEEP) {
            // waves 0-2: park paths that reach p.deep_depth segments (room permitting)
            const uint64_t pm = deep_wave ? 0ull : __ballot(alive && depth >= p.deep_depth);
            if (pm) {
                const uint32_t n = (uint32_t)__popcll(pm);
                uint32_t h0 = 0, n2 = 0;
                if (lane == __builtin_ctzll(pm)) {
                    for (;;) {
                        const uint32_t h = __atomic_load_n(&dq->head, __ATOMIC_RELAXED);
                        const uint32_t t = __atomic_load_n(&dq->tail, __ATOMIC_ACQUIRE);
                        n2 = min(n, kDeepQ - (h - t));
                        h0 = h;
                        if (n2 == 0u) break;
                        uint32_t expect = h;
                        if (__atomic_compare_exchange_n(&dq->head, &expect, h + n2, false, __ATOMIC_ACQ_REL,
                                                        __ATOMIC_RELAXED))
                            break;
                    }
                }
                h0 = __builtin_amdgcn_readlane(h0, __builtin_ctzll(pm));
                n2 = __builtin_amdgcn_readlane(n2, __builtin_ctzll(pm));
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u));
                if ((pm >> lane) & 1ull && rank < n2) {
                    const uint32_t pos = h0 + rank, sl = pos % kDeepQ;
                    dq->st[sl][0] = make_uint4(__float_as_uint(o.x), __float_as_uint(o.y), __float_as_uint(o.z), 0u);
                    dq->st[sl][1] = make_uint4(__float_as_uint(d.x), __float_as_uint(d.y), __float_as_uint(d.z), 0u);
                    dq->st[sl][2] = make_uint4(__float_as_uint(att.x), __float_as_uint(att.y), __float_as_uint(att.z), 0u);
                    dq->st[sl][3] = make_uint4((uint32_t)rng, (uint32_t)(rng >> 32), pix, ls);
                    dq->st[sl][4] = make_uint4(__float_as_uint(pn.x), __float_as_uint(pn.y), __float_as_uint(pn.z),
                                               __float_as_uint(pn.w));
                    dq->meta[sl] = depth | ((uint32_t)pend << 8) | ((uint32_t)pend_metal << 9);
                    __atomic_store_n(&dq->gen[sl], pos / kDeepQ + 1u, __ATOMIC_RELEASE);
                    alive = false;
                    pend = false;  // the pending scatter left with the path
                }
            }
        }
    }
    if constexpr (DEEP) {
        if (!deep_wave && lane == 0) __atomic_fetch_sub(&dq->producers, 1u, __ATOMIC_RELEASE);
    }

    if (p.segments) {
        // wave reductions, one atomic per wave and counter: [0] segments, [1] sphere tests,
        // [2] cluster box tests (lane-level, executed)
        const unsigned long long c[3] = {segs, tests_sph, tests_box};  // widened before the reduction
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            unsigned long long v = c[i];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(p.segments + i, v);
        }
    }
    if (STATS && p.dbg) {
        const uint32_t c[8] = {dbg_iters, dbg_refills, dbg.wave_blocks, dbg.lane_blocks, dbg.wave_roots,
                               dbg.lane_roots, (uint32_t)segs, dbg.wave_member_blocks};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned long long v = c[i];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(p.dbg + i, v);
        }
        if (lane == 0) {
            for (int i = 0; i < 5; ++i) atomicAdd(p.dbg + 8 + i, (unsigned long long)cyc[i]);
            atomicMax(p.dbg + 14, ~t_wave0);  // launch start = ~max(~t) = earliest wave start
        }
        // wave timeline: [16 + 4w] time the queues were found dry (realtime ticks), [17 + 4w] exit,
        // [18 + 4w] loop iterations, [19 + 4w] hardware id << 32 | iterations after dry << 16 |
        // refill rounds; w = wave of the grid. The launch starts at t_wave0 of the earliest wave.
        const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (lane == 0 && w < kDbgWaves) {
            p.dbg[16 + 4 * w] = t_dry ? t_dry : __builtin_amdgcn_s_memrealtime();
            p.dbg[17 + 4 * w] = __builtin_amdgcn_s_memrealtime();
            p.dbg[18 + 4 * w] = dbg_iters;
            p.dbg[19 + 4 * w] = ((unsigned long long)__smid() << 32) | (min(dbg_iters_dry, 65535u) << 16) |
                                min(dbg_refills, 65535u);
        }
    }
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
        uint64_t need = __ballot(!alive);
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
            need = __ballot(!alive);
        }
        if (__ballot(alive) == 0) break;
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
        for (uint32_t w = i; w < k.queue_words; w += gridDim.x * blockDim.x) k.queue_reset[w] = 0u;
    if (i >= k.n_pixels) return;
    f3 acc;
    if (k.first) acc = mk(0.f, 0.f, 0.f);
    else acc = mk(k.acc[3 * i], k.acc[3 * i + 1], k.acc[3 * i + 2]);
    // main.cxx:205 = libstdc++ reduce (<numeric>:443-460): ((c0+c1)+(c2+c3)) per block of 4,
    // blocks in order, then the spp % 4 tail one by one. Passes start on a multiple of 4.
    auto ld = [&](uint32_t s) {
        const float *v = k.slots + ((size_t)s * k.n_pixels + i) * 3u;
        return mk(v[0], v[1], v[2]);
    };
    uint32_t s = 0;
    for (; s < 4u * k.n_blocks; s += 4u) acc = acc + ((ld(s) + ld(s + 1u)) + (ld(s + 2u) + ld(s + 3u)));
    for (; s < k.n_samples; ++s) acc = acc + ld(s);
    if (!k.last) {
        k.acc[3 * i] = acc.x; k.acc[3 * i + 1] = acc.y; k.acc[3 * i + 2] = acc.z;
        return;
    }
    const f3 col = acc / (float)k.spp;  // main.cxx:207
    // output position
    uint32_t x, rr;
    {
        const uint32_t tiled_px = k.tiled_rows * k.W;
        if (i < tiled_px) {
            uint32_t t = i >> 6, w = i & 63u;
            uint32_t ty = t / k.tiles_x, tx = t - ty * k.tiles_x;
            x = (tx << k.tile_lw) + (w & ((1u << k.tile_lw) - 1u));
            rr = (ty << (6u - k.tile_lw)) + (w >> k.tile_lw);
        } else {
            uint32_t jj = i - tiled_px;
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

__global__ __launch_bounds__(256) void epilogue_rgb8_kernel(const float *in, uint8_t *out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double g = (double)(1.f / 2.2f);
    out[i] = (uint8_t)(255.f * (float)pow((double)in[i], g));
}

// ---- launchers (called from rt_host.cpp) ---------------------------------------------
template <int V, bool STATS> static const void *ptr3(int cull, bool deep)
{
    if (deep && cull == 5) return reinterpret_cast<const void *>(&render_kernel<V, 5, STATS, true>);
    if (deep && cull == 0) return reinterpret_cast<const void *>(&render_kernel<V, 0, STATS, true>);
    if (deep) return nullptr;
    if (cull == 1) return reinterpret_cast<const void *>(&render_kernel<V, 1, STATS, false>);
    if (cull == 2) return reinterpret_cast<const void *>(&render_kernel<V, 2, STATS, false>);
    if (cull == 3) return reinterpret_cast<const void *>(&render_kernel<V, 3, STATS, false>);
    if (cull == 4) return reinterpret_cast<const void *>(&render_kernel<V, 4, STATS, false>);
    if (cull == 5) return reinterpret_cast<const void *>(&render_kernel<V, 5, STATS, false>);
    if (cull == 6) return reinterpret_cast<const void *>(&render_kernel<V, 6, STATS, false>);
    if (cull == 7) return reinterpret_cast<const void *>(&render_kernel<V, 7, STATS, false>);
    return reinterpret_cast<const void *>(&render_kernel<V, 0, STATS, false>);
}

static const void *render_ptr(int variant, int cull, bool deep)
{
    switch (variant) {
    case V_EXACT_LDS: return ptr3<V_EXACT_LDS, false>(cull, deep);
    case V_FAST_LDS: return ptr3<V_FAST_LDS, false>(cull, deep);
    case V_EXACT_SCALAR:
        return cull || deep ? nullptr : reinterpret_cast<const void *>(&render_kernel<V_EXACT_SCALAR, 0, false, false>);
    case V_STATS_LDS: return ptr3<V_EXACT_LDS, true>(cull, deep);
    default: return nullptr;
    }
}

hipError_t launch_render(int variant, int cull, const KParams &p, uint32_t grid, hipStream_t stream)
{
    const void *fn = render_ptr(variant, cull, p.deep_depth != 0);
    if (!fn) return hipErrorInvalidValue;
    const size_t lds = (size_t)p.lds_units * 16u;
    void *args[] = {const_cast<KParams *>(&p)};
    return hipLaunchKernel(fn, dim3(grid), dim3(256), args, lds, stream);
}

hipError_t occupancy_render(int variant, int cull, bool deep, int *blocks_per_cu, size_t lds)
{
    const void *fn = render_ptr(variant, cull, deep);
    if (!fn) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 256, lds);
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

hipError_t launch_epilogue(const float *in, uint8_t *out, uint64_t n, hipStream_t stream)
{
    const uint64_t grid = (n + 255u) / 256u;
    hipLaunchKernelGGL(epilogue_rgb8_kernel, dim3((uint32_t)grid), dim3(256), 0, stream, in, out, n);
    return hipGetLastError();
}

} // namespace rt
