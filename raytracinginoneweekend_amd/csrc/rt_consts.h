// rt_consts.h — records and constants shared by the host-only code (rt_host_build.cpp, built
// without HIP, also under the CPU sanitizers), the launcher (rt_host.cpp) and the kernels.
#pragma once
#include <stdint.h>

namespace rt {

// Exact unsigned division by a per-render invariant d (Granlund-Montgomery, "round-up with
// add"): q = (t + ((n - t) >> s1)) >> s2, t = mulhi(n, m), for every 32-bit n; d >= 2: s1 = 1,
// s2 = ceil(log2 d) - 1, m = floor(2^32 (2^ceil(log2 d) - d) / d) + 1; d = 1: m = s1 = s2 = 0
// (t = 0, q = n), so no branch.
struct UDiv {
    uint32_t m, s1, s2;
};

// A lane inside an isolated dielectric sphere (rt_host.cpp isolated_spheres) skips the cluster
// walk when both ends of its segment lie within the ball |p - C|^2 <= fl(fl(r r) kIsoR2Grow)
constexpr float kIsoR2Grow = 1.0201f;
// a dielectric sphere's shortcut word (rt_host.cpp shortcut_words): this bit, then the geo slots
// (+ 1, 0 = none) of its at most two neighbours in bits [0, 15) and [15, 30)
constexpr uint32_t kShortcut = 0x80000000u;
// clusters under one level-2 box (the walk tests a passing box's clusters in pairs). 8: config 3
// frame period 2.548-2.562 vs 2.578-2.596 ms with 4, 6 alike with 4, 12 and 16 slower, 2 +5%
// (profiles/r05/ab/super_clusters.txt)
#ifndef RT_SUPER
#define RT_SUPER 8
#endif
constexpr uint32_t kSuperClusters = RT_SUPER;
static_assert(kSuperClusters % 2 == 0, "clusters are tested in pairs");

} // namespace rt
