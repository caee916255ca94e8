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
__device__ __forceinline__ f3 random_in_unit_sphere(uint64_t &st, uint64_t inc) // raytracer.hxx:32-43
{
    f3 p;
    do {
        float x = canonical(st, inc) * 2.f + -1.f;
        float y = canonical(st, inc) * 2.f + -1.f;
        float z = canonical(st, inc) * 2.f + -1.f;
        p = mk(x, y, z);
    } while (length(p) > 1.f);
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
__device__ __forceinline__ void pixel_of(const KParams &p, uint32_t i, uint32_t &x, uint32_t &rr)
{
    const uint32_t tiled_px = p.tiled_rows * p.W;
    if (i < tiled_px) {
        uint32_t t = i >> 6, w = i & 63u;
        uint32_t ty = t / p.tiles_x, tx = t - ty * p.tiles_x;
        x = tx * 8u + (w & 7u);
        rr = ty * 8u + (w >> 3);
    } else {
        uint32_t j = i - tiled_px;
        rr = j / p.W;
        x = j - rr * p.W;
        rr += p.tiled_rows;
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
    uint32_t wave_blocks, lane_blocks, wave_roots, lane_roots;
};
__device__ __forceinline__ bool first_active_lane()
{
    return (threadIdx.x & 63u) == __builtin_amdgcn_readfirstlane(threadIdx.x & 63u);
}

struct Hit {
    float t;
    uint32_t id;   // original sphere index, 0xffffffff = none
};

template <bool FAST, bool STATS>
__device__ __forceinline__ void test_block8(const float4 *__restrict__ geo, const uint32_t *__restrict__ sidx, uint32_t i,
                                            f3 o, f3 d, float a, Hit &h, Dbg &dbg)
{
    float bq[8], dq[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
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
    float m = fmaxf(fmaxf(fmaxf(dq[0], dq[1]), fmaxf(dq[2], dq[3])), fmaxf(fmaxf(dq[4], dq[5]), fmaxf(dq[6], dq[7])));
    if (m > 0.f) {
        if (STATS) { ++dbg.lane_blocks; if (first_active_lane()) ++dbg.wave_blocks; }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
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
}

// Cluster culling: a lane tests a cluster's spheres only if its ray segment (kMIN, t_best]
// can reach the cluster's AABB grown by a pad that dominates every float error involved
// (1e-3 x (|o|_1 + |C|_1 + |e|_1) against errors below 3e-4 of that), so a
// culled cluster never holds a sphere whose exact candidate could win: same bits.
#define RT_PAD_REL 1e-3f

template <bool FAST, bool CULL, bool STATS>
__device__ __forceinline__ Hit closest_hit(const KParams &p, const float4 *__restrict__ geo,
                                           const uint32_t *__restrict__ sidx, const float4 *__restrict__ clus, f3 o,
                                           f3 d, Dbg &dbg, uint32_t &tests)
{
    const float a = d.x * d.x + d.y * d.y + d.z * d.z;
    Hit h{RT_TMAX, 0xffffffffu};
    for (uint32_t i = 0; i < p.n_always; i += 8) test_block8<FAST, STATS>(geo, sidx, i, o, d, a, h, dbg);
    tests += p.n_always;
    if (CULL) {
        auto safe_rcp = [](float x) {
            return __builtin_amdgcn_rcpf(fabsf(x) < 1e-30f ? copysignf(1e-30f, x) : x);
        };
        const float ix = safe_rcp(d.x), iy = safe_rcp(d.y), iz = safe_rcp(d.z);
        const float oix = o.x * ix, oiy = o.y * iy, oiz = o.z * iz;
        const float aix = fabsf(ix), aiy = fabsf(iy), aiz = fabsf(iz);
        const float opad = RT_PAD_REL * (fabsf(o.x) + fabsf(o.y) + fabsf(o.z));
        for (uint32_t c = 0; c < p.n_clusters; ++c) {
            const float4 c0 = clus[2 * c], c1 = clus[2 * c + 1];   // {C, ex}, {ey, ez, kc, start|count}
            const float pad = opad + c1.z;
            const float hx = (c0.w + pad) * aix, hy = (c1.x + pad) * aiy, hz = (c1.y + pad) * aiz;
            const float tcx = fmaf(c0.x, ix, -oix), tcy = fmaf(c0.y, iy, -oiy), tcz = fmaf(c0.z, iz, -oiz);
            const float tin = fmaxf(fmaxf(tcx - hx, tcy - hy), tcz - hz);
            const float tout = fminf(fminf(tcx + hx, tcy + hy), tcz + hz);
            ++tests;  // box tests are tallied in the high half (see below)
            if (tin <= tout && tout >= 0.5f * RT_TMIN && tin <= h.t * 1.002f) {
                const uint32_t sc = __builtin_amdgcn_readfirstlane(__float_as_uint(c1.w));
                const uint32_t start = sc & 0xffffu, cnt = sc >> 16;
                for (uint32_t i = start; i < start + cnt; i += 8) test_block8<FAST, STATS>(geo, sidx, i, o, d, a, h, dbg);
                tests += cnt << 16;
            }
        }
    }
    return h;
}

// ---- the megakernel ----------------------------------------------------------------------
#ifndef RT_MIN_WAVES_PER_SIMD
#define RT_MIN_WAVES_PER_SIMD 1  // measured: forcing 8 waves (64 VGPRs) spills and runs slower
#endif
template <int V, bool CULL, bool STATS>
__global__ __launch_bounds__(256, RT_MIN_WAVES_PER_SIMD) void render_kernel(const KParams p)
{
    constexpr bool FAST = (V == V_FAST_LDS);
    // Scene blob -> LDS (or read in place from global for the scalar-cache A/B variant):
    // [geo float4 x n_geo][sidx u32 x n_geo, 16-B padded][clusters float4 x 2 x n_clusters]
    extern __shared__ float4 lds_blob[];
    const float4 *blob;
    if constexpr (V == V_EXACT_SCALAR) {
        blob = p.blob;
    } else {
        for (uint32_t i = threadIdx.x; i < p.blob_units; i += blockDim.x) lds_blob[i] = p.blob[i];
        __syncthreads();
        blob = lds_blob;
    }
    const float4 *geo = blob;
    const uint32_t *sidx = reinterpret_cast<const uint32_t *>(blob + p.n_geo);
    const float4 *clus = blob + p.clus_offset;

    const uint32_t lane = threadIdx.x & 63u;
    const float fW = (float)p.W, fH = (float)p.H;

    // wave-uniform cursor over the item space
    uint32_t q = blockIdx.x & 7u, q_tried = 0;
    uint32_t cnext = 0, cend = 0;
    bool exhausted = false;

    // lane state
    bool has_item = false, alive = false;
    uint32_t px = 0, py = 0, pix = 0, slot = 0, s_first = 0, s_count = 0, j = 0;
    f3 o = mk(0.f, 0.f, 0.f), d = o, att = o, pair = o, c2 = o;
    uint32_t depth = 0;
    uint64_t rng = 0;
    unsigned long long segs = 0, tests_sph = 0, tests_box = 0;
    Dbg dbg{0, 0, 0, 0};
    uint32_t dbg_iters = 0, dbg_refills = 0;

    for (;;) {
        // ---- refill items for idle lanes -------------------------------------------
        uint64_t need = __ballot(!has_item);
        if (STATS && need && !exhausted && lane == 0) ++dbg_refills;
        while (need && !exhausted) {
            if (cnext >= cend) {
                uint32_t c = 0;
                if (lane == 0) c = atomicAdd(p.queue_ctr + q, 1u);
                c = __builtin_amdgcn_readfirstlane(c);
                const uint64_t chunk = (uint64_t)q + 8ull * c;
                if (chunk >= p.n_chunks) {
                    q = (q + 1u) & 7u;
                    if (++q_tried == 8u) exhausted = true;
                    continue;
                }
                cnext = (uint32_t)chunk * 64u;
                cend = min(cnext + 64u, p.n_items);
            }
            const uint32_t avail = cend - cnext;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            if (!has_item && rank < avail) {
                const uint32_t I = cnext + rank;
                const uint32_t ls = I / p.n_pixels;
                pix = I - ls * p.n_pixels;
                slot = p.slot_begin + ls;
                uint32_t rr;
                pixel_of(p, pix, px, rr);
                py = p.row_offset + rr * p.row_stride;
                if (slot < p.g4) { s_first = slot * 4u; s_count = 4u; }
                else { s_first = p.g4 * 4u + (slot - p.g4); s_count = 1u; }
                j = 0;
                has_item = true;
            }
            const uint32_t took = min((uint32_t)__popcll(need), avail);
            cnext += took;
            need = __ballot(!has_item);
        }

        // ---- start a sample on lanes that have an item but no live path -------------
        if (has_item && !alive) {
            const uint32_t s = s_first + j;
            const uint64_t key = ((uint64_t)py * p.W + px) * p.spp + s;
            rng = pcg_seed(key, p.inc_data);
            uint64_t rc = pcg_seed(key, p.inc_cam);
            // main.cxx:192-200
            const float u = (float)px / fW;
            const float v = (float)py / fH;
            const float uu = u + canonical(rng, p.inc_data) / fW;
            const float vv = v + canonical(rng, p.inc_data) / fH;
            // camera.hxx:46-57
            const f3 rd = random_in_unit_sphere(rc, p.inc_cam) * p.lens;
            const f3 off = mk(uu * rd.x, vv * rd.y, 0.f);
            const f3 org = mk(p.org[0], p.org[1], p.org[2]);
            o = org + off;
            d = ((mk(p.llc[0], p.llc[1], p.llc[2]) + mk(p.hor[0], p.hor[1], p.hor[2]) * uu) +
                 mk(p.ver[0], p.ver[1], p.ver[2]) * (1.f - vv)) - off;
            if (p.corrected) d = d - org;
            att = mk(1.f, 1.f, 1.f);
            depth = 0;
            alive = true;
        }
        if (__ballot(alive) == 0) break;  // only when the item space is exhausted
        if (STATS && lane == 0) ++dbg_iters;

        // ---- one segment for every live lane ------------------------------------------
        if (alive) {
            bool done = false;
            f3 col = mk(0.f, 0.f, 0.f);
            if (depth >= p.max_depth) {
                done = true;  // main.cxx:74 (only reachable with max_depth == 0)
            } else {
                ++segs;
                uint32_t tally = 0;  // low 16 bits: always-list spheres + box tests; high: member spheres
                const Hit h = closest_hit<FAST, CULL, STATS>(p, geo, sidx, clus, o, d, dbg, tally);
                tests_sph += p.n_always + (tally >> 16);
                tests_box += (tally & 0xffffu) - p.n_always;
                const float t = h.t;
                const uint32_t ib = h.id;
                ++depth;
                if (ib == 0xffffffffu) {
                    // main.cxx:71: background(.5 * unit_direction.y + 1) * attenuation
                    const float tt = .5f * normalize(d).y + 1.f;
                    const f3 bg = mk(1.f, 1.f, 1.f) * (1.f - tt) + mk(.5f, .7f, 1.f) * tt;
                    col = bg * att;
                    done = true;
                } else {
                    const float4 sf = reinterpret_cast<const float4 *>(p.sph_full)[ib];
                    const f3 ctr = mk(sf.x, sf.y, sf.z);
                    const f3 hp = o + d * t;                    // ray::point_at, math.hxx:353
                    const f3 hn = (hp - ctr) / sf.w;            // raytracer.hxx:71
                    const uint32_t mi = p.sph_mat[ib];
                    const float4 md = reinterpret_cast<const float4 *>(p.mat_data)[mi];
                    const uint32_t kind = p.mat_kind[mi];
                    const f3 albedo = mk(md.x, md.y, md.z);
                    bool scattered = true;
                    f3 nd;
                    if (kind == 0u) {                           // lambert, raytracer.hxx:132-141
                        const f3 r = random_in_unit_sphere(rng, p.inc_data);
                        nd = ((hp + hn) + r) - hp;
                    } else if (kind == 1u) {                    // metal, raytracer.hxx:143-156
                        const f3 refl = reflect(normalize(d), hn);
                        const f3 r = random_in_unit_sphere(rng, p.inc_data);
                        nd = refl + r * md.w;
                        scattered = dot(nd, hn) > 0.f;
                    } else {                                    // dielectric, raytracer.hxx:158-194
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
                        if (length(refr) > 0.f) prob = schlick(ri, cosv);
                        nd = canonical(rng, p.inc_data) < prob ? reflect(ud, hn) : refr;
                    }
                    if (!scattered) {
                        done = true;                            // main.cxx:68
                    } else {
                        o = hp;
                        d = nd;
                        att = att * albedo;                     // main.cxx:65
                        if (depth >= p.max_depth) done = true;  // main.cxx:74
                    }
                }
            }
            if (done) {
                // fold the finished sample into its item (main.cxx:205 blocked reduce)
                alive = false;
                bool item_done = false;
                f3 outv = col;
                if (s_count == 1u) {
                    item_done = true;
                } else if (j == 0u) {
                    pair = col;
                } else if (j == 1u) {
                    pair = pair + col;
                } else if (j == 2u) {
                    c2 = col;
                } else {
                    outv = pair + (c2 + col);
                    item_done = true;
                }
                ++j;
                if (item_done) {
                    float *dst = p.slots + ((size_t)(slot - p.slot_begin) * p.n_pixels + pix) * 3u;
                    dst[0] = outv.x;
                    dst[1] = outv.y;
                    dst[2] = outv.z;
                    has_item = false;
                }
            }
        }
    }

    if (p.segments) {
        // wave reductions, one atomic per wave and counter: [0] segments, [1] sphere tests,
        // [2] cluster box tests (lane-level, executed)
        const unsigned long long c[3] = {segs, tests_sph, tests_box};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            unsigned long long v = c[i];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(p.segments + i, v);
        }
    }
    if (STATS && p.dbg) {
        const uint32_t c[7] = {dbg_iters, dbg_refills, dbg.wave_blocks, dbg.lane_blocks, dbg.wave_roots,
                               dbg.lane_roots, (uint32_t)segs};
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            unsigned long long v = c[i];
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) atomicAdd(p.dbg + i, v);
        }
    }
}

// ---- ordered accumulation of the slots, average, optional gamma/u8 --------------------
__global__ __launch_bounds__(256) void accumulate_kernel(const KAccum k)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k.n_pixels) return;
    f3 acc;
    if (k.first) acc = mk(0.f, 0.f, 0.f);
    else acc = mk(k.acc[3 * i], k.acc[3 * i + 1], k.acc[3 * i + 2]);
    for (uint32_t s = 0; s < k.n_local_slots; ++s) {
        const float *v = k.slots + ((size_t)s * k.n_pixels + i) * 3u;
        acc = acc + mk(v[0], v[1], v[2]);
    }
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
            x = tx * 8u + (w & 7u);
            rr = ty * 8u + (w >> 3);
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
static const void *render_ptr(int variant, bool cull)
{
    switch (variant) {
    case V_EXACT_LDS:
        return cull ? reinterpret_cast<const void *>(&render_kernel<V_EXACT_LDS, true, false>)
                    : reinterpret_cast<const void *>(&render_kernel<V_EXACT_LDS, false, false>);
    case V_FAST_LDS:
        return cull ? reinterpret_cast<const void *>(&render_kernel<V_FAST_LDS, true, false>)
                    : reinterpret_cast<const void *>(&render_kernel<V_FAST_LDS, false, false>);
    case V_EXACT_SCALAR:
        return cull ? nullptr : reinterpret_cast<const void *>(&render_kernel<V_EXACT_SCALAR, false, false>);
    case V_STATS_LDS:
        return cull ? reinterpret_cast<const void *>(&render_kernel<V_EXACT_LDS, true, true>)
                    : reinterpret_cast<const void *>(&render_kernel<V_EXACT_LDS, false, true>);
    default:
        return nullptr;
    }
}

hipError_t launch_render(int variant, bool cull, const KParams &p, uint32_t grid, hipStream_t stream)
{
    const void *fn = render_ptr(variant, cull);
    if (!fn) return hipErrorInvalidValue;
    const size_t lds = (variant == V_EXACT_SCALAR) ? 0 : (size_t)p.blob_units * 16u;
    void *args[] = {const_cast<KParams *>(&p)};
    return hipLaunchKernel(fn, dim3(grid), dim3(256), args, lds, stream);
}

hipError_t occupancy_render(int variant, bool cull, int *blocks_per_cu, size_t lds)
{
    const void *fn = render_ptr(variant, cull);
    if (!fn) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 256, lds);
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
