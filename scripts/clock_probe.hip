// clock_probe.hip — the shader clock a wave runs at, against how many waves the GPU runs.
//
// Question (the lone deep launch): the instrumented deep launch shows busy waves
// whose shader-clock cycles (s_memtime) over their life on the 100 MHz realtime clock
// (s_memrealtime) come to 0.7-2.4 GHz when few waves run (the walk shortcut on), and 2.2-2.4 GHz
// when every wave walks (no_shortcut). Here every wave runs the same dependent FMA chain for a
// fixed count and reports cycles and realtime ticks; the launches differ only in how many waves
// run at once (8 .. 8192), and in how long (short runs of ~0.3 ms like the deep launch, long of
// ~3 ms), each launched right after a busy one (as the deep launch follows the main launch).
//
// Build: hipcc --offload-arch=gfx950 -O2 scripts/clock_probe.hip -o scripts/_bin/clock_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void chain(uint32_t iters, float seed, unsigned long long *rec, float *sink)
{
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    float a = seed + threadIdx.x, b = 1.0001f, c = 0.5f;
    for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) a = fmaf(a, b, c);
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t w = blockIdx.x;
    if ((threadIdx.x & 63u) == 0u) {
        rec[2 * w] = c1 - c0;
        rec[2 * w + 1] = r1 - r0;
    }
    if (a == 0.123f) sink[w] = a;
}

static void run(uint32_t waves, uint32_t iters, unsigned long long *drec, float *dsink, const char *label)
{
    hipLaunchKernelGGL(chain, dim3(waves), dim3(64), 0, 0, iters, 1.f, drec, dsink);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * waves);
    hipMemcpy(h.data(), drec, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    std::vector<double> mhz(waves), us(waves);
    for (uint32_t w = 0; w < waves; ++w) {
        mhz[w] = h[2 * w + 1] ? h[2 * w] * 100.0 / h[2 * w + 1] : 0.0;
        us[w] = h[2 * w + 1] / 100.0;
    }
    std::sort(mhz.begin(), mhz.end());
    std::sort(us.begin(), us.end());
    auto q = [&](const std::vector<double> &v, double f) { return v[std::min<size_t>(v.size() - 1, f * v.size())]; };
    std::printf("%-34s waves %5u  clock MHz p0 %6.0f p10 %6.0f p50 %6.0f p90 %6.0f p100 %6.0f   wave us p50 %8.1f\n", label,
                waves, q(mhz, 0), q(mhz, .1), q(mhz, .5), q(mhz, .9), q(mhz, 1), q(us, .5));
}

int main()
{
    unsigned long long *drec;
    float *dsink;
    hipMalloc(&drec, 2 * 65536 * sizeof(unsigned long long));
    hipMalloc(&dsink, 65536 * sizeof(float));
    // warm up
    run(8192, 4000, drec, dsink, "warm-up (8192 waves)");
    for (int rep = 0; rep < 2; ++rep) {
        for (uint32_t waves : {8u, 64u, 256u, 1024u, 2048u, 8192u}) {
            // a busy launch first (every SIMD 8 waves, ~2 ms), then the measured one right after
            run(8192, 4000, drec, dsink, "  busy launch before");
            const uint32_t iters = waves > 1024 ? 8000u * 1024u / waves : 8000u;  // ~0.2-0.3 ms
            char label[64];
            std::snprintf(label, sizeof(label), "after busy, %u waves", waves);
            run(waves, iters, drec, dsink, label);
        }
        for (uint32_t waves : {8u, 256u, 1024u}) {
            char label[64];
            std::snprintf(label, sizeof(label), "long (x10), %u waves", waves);
            run(waves, 80000, drec, dsink, label);
        }
    }
    return 0;
}
