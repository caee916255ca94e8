// Latency of one trapped glass-ball bounce for a lone wave (a diagnostic microbenchmark, not
// product code): the deep launch's chain is ~56 such bounces per path. One
// wave bounces 64 rays inside a glass ball for N iterations with everything but the scene in
// registers, using the product kernel's own device functions (the ball test with its exact
// candidate, the ground's block, the dielectric scatter with Schlick in double and a PCG draw),
// and reports shader cycles per iteration for the full bounce and for its parts.
//   hipcc -std=c++17 -O3 -fno-slp-vectorize --offload-arch=gfx950 -ffp-contract=off -fno-fast-math
//         -I raytracinginoneweekend_amd/csrc scripts/ubench_bounce.hip -o /tmp/ubench_bounce
#include "../raytracinginoneweekend_amd/csrc/rt_kernel.hip"

#include <cstdio>
#include <vector>

namespace ub {
using namespace rt;

// MODE bit 0: the intersection (ball + ground), bit 1: the dielectric scatter
struct UParams {
    const float4 *g_geo;
    const uint32_t *g_sidx;
    int iters;
    float *out;
    unsigned long long *cyc;
    uint32_t fast_roots, n_always, max_depth;
};
// MODE bit 2: three kernel parameters re-read each iteration through an opaque kernarg pointer
// (the product loop's way of holding no SGPRs across iterations)
template <int MODE>
__global__ __launch_bounds__(64) void bounce(const UParams P)
{
    const float4 *g_geo = P.g_geo;
    const uint32_t *g_sidx = P.g_sidx;
    const int iters = P.iters;
    float *out = P.out;
    unsigned long long *cyc = P.cyc;
    typedef const __attribute__((address_space(4))) UParams *up_t;
    const up_t up_base = (up_t)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ float4 geo[2];
    __shared__ uint32_t sidx[2];
    if (threadIdx.x < 2) {
        geo[threadIdx.x] = g_geo[threadIdx.x];
        sidx[threadIdx.x] = g_sidx[threadIdx.x];
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x;
    const float4 S = geo[1];  // the ball: centre, r^2
    const float sr = 0.3f;    // its signed radius
    const float4 dcs = make_float4(1.f / 1.5f, (1.f - 1.5f) / (1.f + 1.5f), (1.f - 1.f / 1.5f) / (1.f + 1.f / 1.5f), 0.f);
    f3 o = mk(S.x + 0.01f * (float)(lane & 7), S.y + 0.01f * (float)(lane >> 3), S.z);
    f3 d = mk(0.3f + 0.001f * lane, -0.2f, 1.f);
    f3 att = mk(1.f, 1.f, 1.f);
    uint64_t rng = 0x853c49e6748fea9bull + lane;
    const uint64_t inc = 0xda3e39cb94b95bdbull;
    Dbg dbg{};
    float tsum = 0.f;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        uint32_t fr = 1u, nalw = 1u, mdep = 1000000u;
        if (MODE & 4) {
            up_t up = up_base;
            asm volatile("" : "+s"(up));
            fr = up->fast_roots;
            nalw = up->n_always;
            mdep = up->max_depth;
        }
        if ((uint32_t)it >= mdep) break;
        const float a = d.x * d.x + d.y * d.y + d.z * d.z;
        const RayDiv rd = ray_div(a, ballot(true), fr);
        float t = 0.5f;
        if (MODE & 1) {
            bool inside;
            Hit h{hint_candidate<false>(true, S, 1u | kShortcut, 0u, geo, sidx, o, d, rd, 1u, inside)};
            if (nalw == 1u) test_block8<false, false, 1>(geo, sidx, 0, o, d, rd, h, dbg);
            t = h.t();
            if (!(t < 1e30f)) t = 0.5f;  // keep the loop going for lanes that left the ball
        }
        tsum += t;
        if (MODE & 2) {
            const f3 hp = o + d * t;
            const f3 dv = hp - mk(S.x, S.y, S.z);
            f3 hn;
            if (all_lanes_min_abs_ok(dv)) hn = div3_short(dv, sr);
            else hn = dv / sr;
            o = hp;
            f3 ud;
            if (rd.fd != 0u && all_lanes_min_abs_ok(d)) ud = div3_short(d, sqrt_scaled(a));
            else ud = normalize(d);
            const f3 rf = reflect(ud, hn);
            f3 outward = mk(-hn.x, -hn.y, -hn.z);
            float ri = 1.5f, xs = dcs.y;
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
            d = canonical(rng, inc) < prob ? rf : refr;
            if (!(d.x == d.x)) d = mk(0.3f, -0.2f, 1.f);
            // stay near the ball (a benchmark, not a path)
            o = mk(S.x + 0.5f * (o.x - S.x), S.y + 0.5f * (o.y - S.y), S.z + 0.5f * (o.z - S.z));
        } else {
            d = mk(d.y, d.z, d.x + 1e-3f);  // a dependent update
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[lane] = tsum + o.x + d.x + att.x + (float)dbg.wave_blocks;
    if (lane == 0) cyc[0] = t1 - t0;
}
} // namespace ub

int main()
{
    // the ground (index 0) and a small glass ball (index 1), as geo entries {C, fl(r r)}
    std::vector<float4> geo = {make_float4(0.f, -1000.f, 0.f, 1000.f * 1000.f), make_float4(4.f, 0.3f, 1.f, 0.3f * 0.3f)};
    std::vector<uint32_t> sidx = {0u, 1u};
    float4 *dg;
    uint32_t *ds;
    float *dout;
    unsigned long long *dc;
    (void)hipMalloc(&dg, sizeof(float4) * 2);
    (void)hipMalloc(&ds, sizeof(uint32_t) * 2);
    (void)hipMalloc(&dout, 64 * sizeof(float));
    (void)hipMalloc(&dc, sizeof(unsigned long long));
    (void)hipMemcpy(dg, geo.data(), sizeof(float4) * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(ds, sidx.data(), sizeof(uint32_t) * 2, hipMemcpyHostToDevice);
    const int iters = 4096;
    ub::UParams up{dg, ds, iters, dout, dc, 1u, 1u, 1000000u};
    auto run = [&](auto kern, const char *name) {
        unsigned long long c = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, up);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
        }
        std::printf("%-28s %8.0f cycles per iteration (one wave alone)\n", name, (double)c / iters);
    };
    run(ub::bounce<1>, "intersection (ball+ground)");
    run(ub::bounce<2>, "dielectric scatter");
    run(ub::bounce<3>, "full bounce");
    run(ub::bounce<0>, "empty loop");
    run(ub::bounce<4>, "empty loop + 3 kernarg re-reads");
    run(ub::bounce<7>, "full bounce + 3 kernarg re-reads");
    // the same bounce on 1024 waves at once (one per SIMD), as in a deep launch
    {
        unsigned long long c = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(ub::bounce<3>, dim3(1024), dim3(64), 0, 0, up);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
        }
        std::printf("%-28s %8.0f cycles per iteration (1024 waves, wave 0 of block 0)\n", "full bounce, 1024 waves", (double)c / iters);
    }
    return 0;
}
