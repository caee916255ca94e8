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

// ---- tile classes of a pass ---------------------------------------------
// What the classifier needs of a culled scene: the always-tested spheres, the box of every
// non-empty cluster and the box over all of them (centre C, half-extent E), the kernel's pad.
struct scene_geom {
    std::vector<rt_sphere> always;
    std::vector<float> boxes;  // per non-empty cluster: C[3], E[3]
    float root[6] = {0.f, 0.f, 0.f, -1.f, -1.f, -1.f};
    bool has_root = false;
    float clus_pad = 0.f;
};
scene_geom scene_geometry(const rt_sphere *s, const blob_t &b);
// The 64-pixel blocks of a pass's pixel enumeration (tiles of 2^tile_lw x 64/2^tile_lw over
// tiled_rows, then row-major blocks of the remaining rows) in dealing order: `lead` blocks first
// (a primary ray of the tile can meet a cluster's padded box: the tiles whose paths can enter a
// glass ball on their first or second segment), then the others, then `sky` blocks, whose every
// primary ray is PROVEN to meet no sphere (interval arithmetic over the tile's rays, with
// margins far above every float error of the kernel's tests). perm[i] = the natural block of
// dealing block i. Empty perm: the pass keeps its natural order (pixels not in whole blocks).
struct tile_order {
    std::vector<uint32_t> perm;
    uint32_t n_lead = 0, n_sky = 0;
};
tile_order classify_tiles(const rt_camera &cam, uint32_t W, uint32_t H, uint32_t row_offset, uint32_t row_stride,
                          uint32_t num_rows, uint32_t tile_lw, const scene_geom &g, bool sky_only = false);

rt::UDiv make_udiv(uint32_t d);
bool exact_by_reciprocal(float b);

} // namespace rthost
