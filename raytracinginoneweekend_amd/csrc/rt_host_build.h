// rt_host_build.h — the host-only half of the library (rt_host_build.cpp): error reporting,
// options, the reference's camera and scene constructors, the scene blob and cluster builder,
// the walk-shortcut proofs, exact-division checks and the PPM writer. No HIP: this half is also
// built with -fsanitize=address,undefined / thread for the CPU sanitizer runs (tests/sanitize).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_consts.h"

namespace rthost {

extern thread_local std::string g_error;
int fail(int code, const std::string &msg);

constexpr uint64_t kMaxSlotsBytes = 1ull << 31;  // slot workspace per pass (2 GiB)
// (the kernel forms a slot index sample * n_pixels + pixel in 32 bits)
static_assert(kMaxSlotsBytes / 12 < (1ull << 32), "slot index width");
// internal render streams for frames in flight (rt_options.render_streams, 2..kMaxBufs), and
// workspaces: rt_options.workspaces_per_stream (1..2) per stream, at most kMaxWs
constexpr uint32_t kMaxBufs = 8;
constexpr uint32_t kMaxWs = 2 * kMaxBufs + 1;  // + the lone passes' own workspace (sample pairs, rt_host.cpp)

rt_options library_defaults();
int check_options(const rt_options &o);
// the process default (rt_set_default_options / RT_OPTIONS)
int default_options(rt_options &out);

// ---- scene blob: always-tested list + spatial clusters -------------------
struct blob_t {
    std::vector<float> data;  // 16-byte units
    uint32_t n_geo = 0, n_always = 0, n_clusters = 0, clus_offset = 0, n_clusters_real = 0;
    uint32_t n_supers = 0, supers_offset = 0, shade_offset = 0;
    float clus_pad = 0.f;
    std::vector<uint32_t> always;  // sphere indices tested on every segment (not clustered)
};
blob_t build_blob(const rt_sphere *s, uint32_t n, bool clustered, uint32_t cluster_max);
std::vector<uint32_t> shortcut_words(const rt_sphere *s, uint32_t n, const rt_material *m, const blob_t &b,
                                     bool nb_off);

rt::UDiv make_udiv(uint32_t d);
bool exact_by_reciprocal(float b);

} // namespace rthost
