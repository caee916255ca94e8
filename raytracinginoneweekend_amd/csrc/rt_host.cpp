// rt_host.cpp — host side of the C-ABI (include/rt_api.h): scene/camera construction that
// mirrors the reference's host code bit for bit, device scene upload, pass planning and the
// render entry points that replace `cuda_impl` (src/main.cxx:18, src/CUDA/cuda_impl.cu:384).
//
// Compiled with -ffp-contract=off: the camera basis and the huge-scene generator must round
// exactly like the reference's (g++, x86-64 SSE, no contraction).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_device.h"

namespace rt {
hipError_t launch_render(int variant, int cull, const KParams &p, uint32_t grid, hipStream_t stream);
hipError_t occupancy_render(int variant, int cull, int *blocks_per_cu, size_t lds);
hipError_t launch_accumulate(const KAccum &k, hipStream_t stream);
hipError_t launch_compat(const KCompat &k, uint32_t grid, hipStream_t stream);
hipError_t launch_wave_gen(const KWave &w, hipStream_t stream);
hipError_t launch_wave_bounce(int cull, const KWave &w, uint32_t grid, hipStream_t stream);
hipError_t occupancy_wave_bounce(int cull, int *blocks_per_cu, size_t lds);
hipError_t occupancy_compat(int *blocks_per_cu);
hipError_t launch_epilogue(const float *in, uint8_t *out, uint64_t n, hipStream_t stream);
} // namespace rt

namespace {

thread_local std::string g_error;

int fail(int code, const std::string &msg)
{
    g_error = msg;
    return code;
}

#define RT_HIP(call)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(RT_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ---- host vector math in the reference's evaluation order (src/math.hxx) ------------
struct hv { float x, y, z; };
hv operator+(hv a, hv b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
hv operator-(hv a, hv b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
hv operator*(hv a, float s) { return {a.x * s, a.y * s, a.z * s}; }
float hlen(hv a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
hv hnorm(hv a)
{
    float l = hlen(a);
    return std::fabs(l) > FLT_MIN ? hv{a.x / l, a.y / l, a.z / l} : a;
}
hv hcross(hv l, hv r) { return {l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x}; }

constexpr uint64_t kMaxSlotsBytes = 1ull << 31;  // slot workspace per pass (2 GiB)
// (the kernel forms a slot index sample * n_pixels + pixel in 32 bits)
static_assert(kMaxSlotsBytes / 12 < (1ull << 32), "slot index width");
// 2 x 8 queue lines, 2 x 4 u64 segment counters, then the compat kernel's pixel counter
// internal render streams for frames in flight (RT_PIPELINE = 2..kMaxBufs), and workspaces:
// RT_WS_PER_STREAM (1..2) per stream, at most kMaxWs
constexpr uint32_t kMaxBufs = 8;
constexpr uint32_t kMaxWs = 2 * kMaxBufs;
constexpr uint32_t kDeepSplitDefault = 8;  // RT_DEEP_SPLIT
// counters: [kMaxWs][8 queues x kQueueStride], then [kMaxWs][4] u64 segment counters, then
// the compat kernel's counter
constexpr size_t kSegWords = kMaxWs * 8 * rt::kQueueStride;
constexpr size_t kCompatCtr = kSegWords + kMaxWs * 8 + 16;
constexpr size_t kCtrWords = kCompatCtr + rt::kQueueStride;

// RT_WAVE_QUEUE_RAYS: rays per chunk of the wavefront variant (default 2^25: 2 x 1.7 GB queues)
uint64_t wave_queue_env()
{
    const char *e = std::getenv("RT_WAVE_QUEUE_RAYS");
    const unsigned long long v = e ? std::strtoull(e, nullptr, 10) : 0ull;
    return v ? std::max<uint64_t>(v, 64) : (1ull << 25);
}

// RT_SLOT_BUDGET_BYTES lowers the per-pass slot workspace (tests force multi-pass renders).
uint64_t slot_budget()
{
    const char *e = std::getenv("RT_SLOT_BUDGET_BYTES");
    const unsigned long long v = e ? std::strtoull(e, nullptr, 10) : 0ull;
    return v ? std::min<uint64_t>(v, kMaxSlotsBytes) : kMaxSlotsBytes;
}

// Items per queue grab (RT_CHUNK_ITEMS for A/B: a multiple of 64 in [64, 8192]); bigger
// chunks mean fewer cross-XCD atomics, smaller ones a finer end-of-launch balance.
uint32_t chunk_items()
{
    const char *e = std::getenv("RT_CHUNK_ITEMS");
    const unsigned long v = e ? std::strtoul(e, nullptr, 10) : 0ul;
    return v >= 64 && v <= 8192 && v % 64 == 0 ? static_cast<uint32_t>(v) : 512u;
}

// Item dealing (default guided, K = RT_GUIDED_K, default 6): each queue's chunks shrink
// geometrically from 1/K of its remaining share per wave down to 128 items — few queue
// atomics, big coherent chunks for most of the launch, small ones at its end. Config 3 frame
// stream: K = 6 3.93 ms/frame with single-frame latency unchanged (5.3-5.4 ms); K = 4
// 3.89-3.92 but 6.2 ms latency; the fixed scheme (RT_SCHED=fixed: RT_CHUNK_ITEMS chunks, the
// last RT_TAIL_PCT % in 64s) 4.39 ms at 512/8%, 3.96 at 2048/2% (5.7 ms latency).
// Round 3: a pass issued while no other render runs (a lone frame) deals with K = 12 — its end
// is not hidden by other launches, and smaller last chunks even it out (config 3 lone frame
// 3.37-3.45 vs 3.55-3.59 ms, frame stream alike at K = 6/9/12; profiles/r03/ab/guided_k.txt).
float guided_l2b(uint32_t total_waves, bool in_flight)
{
    const char *e = std::getenv("RT_SCHED");
    if (e && std::strcmp(e, "fixed") == 0) return 0.f;
    const char *ke = std::getenv("RT_GUIDED_K");
    const double k = ke && *ke ? std::max(0.25, std::atof(ke)) : (in_flight ? 6.0 : 12.0);
    const double wq = std::max(1.0, total_waves / 8.0);
    const double beta = std::max(1.0 - 1.0 / (k * wq), 1.0 / (1 << 20));
    return static_cast<float>(std::log2(beta));
}

// log2 of the tile width (RT_TILE_LW=3..6 for A/B; default 3 = 8x8 tiles). Tiles whose image
// footprint stays near square for strided rows (16x4 at stride 2-4, 32x2 at 5-8) were not
// faster: row shares of config 3 at N = 8: 8x8 0.61-0.62 ms, 32x2 0.62, 64x1 0.66; N = 4:
// 8x8 1.08-1.10, 16x4 1.10, 32x2 1.14; N = 2: 8x8 1.99, 16x4 2.02-2.05.
uint32_t tile_lw_for(uint32_t width, uint32_t stride)
{
    (void)stride;
    const char *e = std::getenv("RT_TILE_LW");
    uint32_t lw = 3u;
    if (e && *e) lw = static_cast<uint32_t>(std::clamp<long>(std::strtol(e, nullptr, 10), 3, 6));
    while (lw > 3 && width % (1u << lw)) --lw;  // the tile width must divide the row
    return lw;
}

// Workgroups per CU of a render launch. A launch that finds no other render in flight (a
// single frame, the first of a stream) takes the occupancy: the lowest latency. One issued
// while earlier renders still run takes half of it, (occ + 1) / 2, so consecutive launches run
// side by side instead of each waiting for the previous one's workgroups to retire, and each
// one's drain overlaps the others' bulk: half the occupancy, and for passes of at most
// kShortPassItems samples with n render streams ceil(occ / (n - 1)) (4 streams: a third).
// Measured with 3 streams (occupancy 6, in-flight grid 3 / 4 / 6):
// config 3 frame stream 3.80-3.92 / 3.81-3.88 / 3.89-3.93 ms; 2-way row share 1.97-2.01 /
// 2.03-2.05 / 2.08; 8-way row share 0.63 / 0.66 / 0.68 (2: 0.66); configs 4 and 5 equal.
// With 4 streams (GPU_MAX_HW_QUEUES=8): grid 2: config 3 3.83-3.84 ms, 8-way 0.60-0.61; grid
// 3: 3.84-3.86, 0.65 — but config 3 with the corrected camera (7 segments per primary, 29 ms
// frames) 32.0-34.3 ms at grid 2 vs 29.8 at grid 3 (28.8 with 2 streams and full grids), so
// the third applies to short passes only. RT_GRID_WG_PER_CU=n sets the in-flight grid (A/B).
constexpr uint64_t kShortPassItems = 32ull << 20;
int grid_wg_per_cu(int occ, bool in_flight, uint32_t streams, uint64_t pass_items)
{
    if (!in_flight) return occ;
    const char *e = std::getenv("RT_GRID_WG_PER_CU");
    const long v = e && *e ? std::strtol(e, nullptr, 10) : 0;
    if (v > 0) return std::min<int>(occ, static_cast<int>(v));
    const int others = pass_items <= kShortPassItems ? std::max(1, static_cast<int>(streams) - 1)
                                                     : std::min(2, std::max(1, static_cast<int>(streams) - 1));
    return std::max(1, (occ + others - 1) / others);
}

// Share of a launch's items dealt in 64-item chunks at its end (RT_TAIL_PCT for A/B, 0-100).
uint32_t tail_pct()
{
    const char *e = std::getenv("RT_TAIL_PCT");
    const unsigned long v = e && *e ? std::strtoul(e, nullptr, 10) : 8ul;
    return v <= 100 ? static_cast<uint32_t>(v) : 8u;
}

} // namespace

struct rt_scene {
    int device = 0;
    uint32_t n_spheres = 0, n_materials = 0;
    // scene blobs: [0] every sphere in index order (brute force), [1] big
    // spheres always tested + spatial clusters
    float *blob[2] = {nullptr, nullptr};
    uint32_t blob_units[2] = {0, 0}, n_geo[2] = {0, 0}, n_always[2] = {0, 0}, n_clusters[2] = {0, 0},
             clus_offset[2] = {0, 0};
    float clus_pad[2] = {0.f, 0.f};
    uint32_t n_supers[2] = {0, 0}, supers_offset[2] = {0, 0};
    uint32_t shade_offset[2] = {0, 0};
    bool in_fast_range = false;  // every sphere within 2^19 of the origin, radii >= 2^-40 (short exact forms)
    // workspaces: consecutive render passes (of one frame or of consecutive frames) rotate over
    // internal streams xs[b] and workspaces slots[b], so a pass renders while the caller stream
    // still accumulates the previous ones
    float *slots[kMaxWs] = {};
    size_t slots_bytes[kMaxWs] = {};
    float *acc = nullptr;
    size_t acc_bytes = 0;
    // deep-path split: per workspace, the pixel flags (a byte per pixel, at the front) and then
    // the deep queue (rt::DeepQueue); deep_clean = leading bytes known to be zero (every pass's
    // accumulation clears the flags it set, so only a larger pixel count needs a memset)
    void *deep[kMaxWs] = {};
    size_t deep_bytes[kMaxWs] = {}, deep_clean[kMaxWs] = {};
    // deep-queue overflow reports (pinned host memory written by accumulate_kernel, one word per
    // workspace) and the camera keys they named, with the call that last reported each: renders
    // with such a camera are not split for kDeepOffCalls calls; at most kDeepOffKeys keys (LRU)
    unsigned long long *deep_over = nullptr, *deep_over_dev = nullptr;
    static constexpr size_t kDeepOffKeys = 8;
    static constexpr uint64_t kDeepOffCalls = 256;
    std::vector<std::pair<unsigned long long, uint64_t>> deep_off;
    void *wq = nullptr;  // RT_FLAG_WAVEFRONT: two ray queues and their counters
    size_t wq_bytes = 0;
    int occ_wave[2] = {-1, -1};  // wave_bounce_kernel blocks per CU [culled], -1 = unknown
    uint32_t *queue_ctr = nullptr;  // kCtrWords: queue and segment counters (layout at kCtrWords)
    hipStream_t xs[kMaxBufs] = {};
    hipEvent_t ev_done[kMaxWs] = {}, ev_free[kMaxWs] = {};
    hipEvent_t ev_main[kMaxWs] = {};  // split passes: after the main launch (created on first use)
    bool free_valid[kMaxWs] = {};
    // queue/segment counters of workspace b not known to be zero (set while a render using
    // them is enqueued, cleared once the accumulation that resets them is enqueued after it)
    bool ctr_dirty[kMaxWs];
    rt_scene() { std::fill(std::begin(ctr_dirty), std::end(ctr_dirty), true); }
    uint32_t next_buf = 0;  // workspace of the next render pass
    int last_ws = -1;       // workspace of the last render pass issued (its ev_done), -1 = none
    // the caller stream of the previous call and an event after the last work enqueued on it:
    // a call on another stream first waits for it, so the shared accumulation buffer, the
    // compat counter and (RT_PIPELINE=0) the workspaces are never used by two streams at once
    hipStream_t last_stream = nullptr;
    hipEvent_t ev_tail = nullptr;
    bool tail_valid = false;
    int cu_count = 0;
    int occ[4][2][2];  // [variant][culled][shade records in LDS] blocks per CU, -1 = unknown
    unsigned long long *dbg = nullptr;  // diagnostic counters (RT_DEBUG_STATS=1)
    uint32_t dbg_waves = 0;             // waves of the last instrumented launch
    size_t max_lds = 0;
    // ring of (start, end) events bracketing the render kernels of each rt_render_device call
    static constexpr uint32_t kRing = 256;
    std::vector<hipEvent_t> ev_begin, ev_end;
    uint64_t calls = 0;
};

extern "C" {

int rt_version(void) { return RT_API_VERSION; }

const char *rt_last_error(void) { return g_error.c_str(); }

int rt_device_count(int *count)
{
    if (!count) return fail(RT_ERR_INVALID, "rt_device_count: null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return RT_OK;
}

// raytracer::camera ctor, src/camera.hxx:24-44.
int rt_camera_init(const float position[3], const float lookat[3], const float up[3], float aspect,
                   float vfov_degrees, float aperture, float focus_distance, uint32_t mode, rt_camera *out)
{
    if (!position || !lookat || !up || !out) return fail(RT_ERR_INVALID, "rt_camera_init: null argument");
    if (mode > RT_CAMERA_CORRECTED) return fail(RT_ERR_INVALID, "rt_camera_init: bad mode");
    const hv P{position[0], position[1], position[2]}, L{lookat[0], lookat[1], lookat[2]}, U{up[0], up[1], up[2]};
    const float theta = (vfov_degrees * static_cast<float>(0.01745329251994329576923690768489)) / 2.f; // math.hxx:8-13
    const float height = std::tan(theta);
    const float width = height * aspect;
    const hv w = hnorm(P - L);
    const hv u = hnorm(hcross(U, w));
    const hv v = hnorm(hcross(w, u));
    const hv llc = P - ((u * width + v * height) + w) * focus_distance;
    const hv hor = ((u * width) * focus_distance) * 2.f;
    const hv ver = ((v * height) * focus_distance) * 2.f;
    rt_camera c{};
    c.origin[0] = P.x; c.origin[1] = P.y; c.origin[2] = P.z;
    c.lower_left_corner[0] = llc.x; c.lower_left_corner[1] = llc.y; c.lower_left_corner[2] = llc.z;
    c.horizontal[0] = hor.x; c.horizontal[1] = hor.y; c.horizontal[2] = hor.z;
    c.vertical[0] = ver.x; c.vertical[1] = ver.y; c.vertical[2] = ver.z;
    c.lens_radius = aperture / 2.f;
    c.mode = mode;
    *out = c;
    return RT_OK;
}

// src/main.cxx:179-183
int rt_camera_cuda(uint32_t width, uint32_t height, rt_camera *out)
{
    // cuda_impl.cu:371-375: position 0, look (0, 0, -1), up y, vFOV 88, aperture .0625, focus 1;
    // camera::ray has no lens offset under CUDA_IMPL (camera.hxx:48-50), and with the origin at
    // 0 the missing "- origin" does not matter
    if (!width || !height) return fail(RT_ERR_INVALID, "rt_camera_cuda: zero size");
    const float pos[3] = {0.f, 0.f, 0.f}, look[3] = {0.f, 0.f, -1.f}, up[3] = {0.f, 1.f, 0.f};
    return rt_camera_init(pos, look, up, static_cast<float>(width) / static_cast<float>(height), 88.f, .0625f, 1.f,
                          RT_CAMERA_REFERENCE, out);
}

int rt_camera_default(uint32_t width, uint32_t height, uint32_t mode, rt_camera *out)
{
    if (!width || !height) return fail(RT_ERR_INVALID, "rt_camera_default: zero size");
    const float pos[3] = {-4.f, 3.2f, 5.f}, look[3] = {0.f, 1.f, 0.f}, up[3] = {0.f, 1.f, 0.f};
    const float focus = hlen(hv{pos[0], pos[1], pos[2]} - hv{look[0], look[1], look[2]});
    return rt_camera_init(pos, look, up, static_cast<float>(width) / static_cast<float>(height), 42.f, 0.0625f,
                          focus, mode, out);
}

} // extern "C"

namespace {

struct scene_builder {
    std::vector<rt_sphere> s;
    std::vector<rt_material> m;
    void mat(uint32_t kind, float r, float g, float b, float param) { m.push_back({kind, {r, g, b}, param}); }
    void sph(float x, float y, float z, float radius, uint32_t mi) { s.push_back({{x, y, z}, radius, mi}); }
    void simple()  // src/main.cxx:120-129
    {
        mat(RT_LAMBERT, static_cast<float>(.1), static_cast<float>(.2), static_cast<float>(.5), 0.f);
        mat(RT_METAL, static_cast<float>(.8), static_cast<float>(.6), static_cast<float>(.2), 0.f);
        mat(RT_DIELECTRIC, 1.f, 1.f, 1.f, 1.5f);
        mat(RT_LAMBERT, static_cast<float>(.64), static_cast<float>(.8), static_cast<float>(.0), 0.f);
        sph(0.f, 1.f, 0.f, 1.f, 0);
        sph(0.f, -1000.125f, 0.f, 1000.f, 3);
        sph(2.f, 1.f, 0.f, 1.f, 1);
        sph(-2.f, 1.f, 0.f, 1.f, 2);
        sph(-2.f, 1.f, 0.f, -.99f, 2);
    }
    // src/main.cxx:131-177 (namespace typo fixed). Draw order: type, center.x, center.z, then
    // the material's draws; a type-3 sphere pushes no material, so it shares the index of the
    // next pushed one and trailing ones are resolved by default materials (lambert, albedo 1).
    void cuda_variant()  // src/CUDA/cuda_impl.cu:425-437
    {
        mat(RT_LAMBERT, static_cast<float>(.1), static_cast<float>(.2), static_cast<float>(.5), 0.f);
        mat(RT_METAL, static_cast<float>(.8), static_cast<float>(.6), static_cast<float>(.2), 0.f);
        mat(RT_DIELECTRIC, 1.f, 1.f, 1.f, 1.5f);
        mat(RT_LAMBERT, static_cast<float>(.64), static_cast<float>(.8), static_cast<float>(.0), 0.f);
        sph(0.f, 0.f, -1.f, .5f, 0);
        sph(0.f, -100.5f, -1.f, 100.f, 3);
        sph(1.f, 0.f, -1.f, .5f, 1);
        sph(-1.f, 0.f, -1.f, .5f, 2);
        sph(-1.f, 0.f, -1.f, -.499f, 2);
    }
    void huge(uint32_t seed)
    {
        simple();
        std::mt19937 gen{seed};
        std::uniform_int_distribution<int> rd_int{0, 3};
        std::uniform_real_distribution<float> rd_real{0.f, 1.f};
        for (int a = -11; a < 11; ++a) {
            for (int b = -11; b < 11; ++b) {
                const int type = rd_int(gen);
                const float cx = .9f * rd_real(gen) + static_cast<float>(a);
                const float cz = .9f * rd_real(gen) + static_cast<float>(b);
                if (hlen(hv{cx, .2f, cz} - hv{0.f, 1.f, 0.f}) < 1.f) continue;
                sph(cx, .2f, cz, .2f, static_cast<uint32_t>(m.size()));
                if (type == 0) {
                    const float r = rd_real(gen), g = rd_real(gen), bb = rd_real(gen);
                    mat(RT_LAMBERT, r, g, bb, 0.f);
                } else if (type == 1) {
                    const float r = rd_real(gen), g = rd_real(gen), bb = rd_real(gen);
                    const float rough = .5f * rd_real(gen);
                    mat(RT_METAL, r, g, bb, rough);
                } else if (type == 2) {
                    const float r = rd_real(gen), g = rd_real(gen), bb = rd_real(gen);
                    mat(RT_DIELECTRIC, r, g, bb, 1.5f);
                }
            }
        }
        uint32_t need = 0;
        for (auto &x : s) need = std::max(need, x.material + 1u);
        while (m.size() < need) mat(RT_LAMBERT, 1.f, 1.f, 1.f, 0.f);
    }
    int emit(rt_sphere *spheres, uint32_t sphere_cap, uint32_t *n_spheres, rt_material *materials,
             uint32_t material_cap, uint32_t *n_materials) const
    {
        if (n_spheres) *n_spheres = static_cast<uint32_t>(s.size());
        if (n_materials) *n_materials = static_cast<uint32_t>(m.size());
        if (spheres) {
            if (sphere_cap < s.size()) return fail(RT_ERR_CAPACITY, "scene: sphere buffer too small");
            std::memcpy(spheres, s.data(), s.size() * sizeof(rt_sphere));
        }
        if (materials) {
            if (material_cap < m.size()) return fail(RT_ERR_CAPACITY, "scene: material buffer too small");
            std::memcpy(materials, m.data(), m.size() * sizeof(rt_material));
        }
        return RT_OK;
    }
};

// ---- scene blob: always-tested list + spatial clusters -------------------
struct blob_t {
    std::vector<float> data;  // 16-byte units
    uint32_t n_geo = 0, n_always = 0, n_clusters = 0, clus_offset = 0, n_clusters_real = 0;
    uint32_t n_supers = 0, supers_offset = 0, shade_offset = 0;
    float clus_pad = 0.f;
    std::vector<uint32_t> always;  // sphere indices tested on every segment (not clustered)
};

constexpr float kPadRel = 1e-3f;      // must match RT_PAD_REL in rt_kernel.hip
// Spheres per cluster: 16 (two blocks of 8); RT_CLUSTER_SIZE (4..64, multiple of 4) for A/B,
// read when a scene is created.
uint32_t cluster_max()
{
    const char *e = std::getenv("RT_CLUSTER_SIZE");
    const unsigned long v = e && *e ? std::strtoul(e, nullptr, 10) : 16ul;
    return v >= 4 && v <= 64 && v % 4 == 0 ? static_cast<uint32_t>(v) : 16u;
}

void split_clusters(const rt_sphere *s, std::vector<uint32_t> ids, std::vector<std::vector<uint32_t>> &out)
{
    const uint32_t kClusterMax = cluster_max();
    if (ids.size() <= kClusterMax) {
        out.push_back(std::move(ids));
        return;
    }
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i : ids)
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], s[i].center[a]);
            hi[a] = std::max(hi[a], s[i].center[a]);
        }
    int ax = 0;
    for (int a = 1; a < 3; ++a)
        if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
    // split at a multiple of the cluster size so leaves come out full
    const size_t half = ((ids.size() / 2 + kClusterMax - 1) / kClusterMax) * kClusterMax;
    const size_t mid = std::min(half, ids.size() - 1);
    std::nth_element(ids.begin(), ids.begin() + mid, ids.end(), [&](uint32_t x, uint32_t y) {
        return s[x].center[ax] < s[y].center[ax] || (s[x].center[ax] == s[y].center[ax] && x < y);
    });
    std::vector<uint32_t> left(ids.begin(), ids.begin() + mid), right(ids.begin() + mid, ids.end());
    split_clusters(s, std::move(left), out);
    split_clusters(s, std::move(right), out);
}

blob_t build_blob(const rt_sphere *s, uint32_t n, bool clustered)
{
    // three classes by |r| against the median: huge (> 64x, e.g. the ground) are tested on
    // every segment; big (> 4x) and small are clustered separately so that one big sphere
    // does not inflate the boxes of the small ones
    std::vector<uint32_t> always, big, small;
    if (clustered && n >= 2 * cluster_max()) {
        std::vector<float> r(n);
        for (uint32_t i = 0; i < n; ++i) r[i] = std::fabs(s[i].radius);
        std::vector<float> sorted = r;
        std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
        const float med = sorted[n / 2];
        for (uint32_t i = 0; i < n; ++i) {
            const bool finite = std::isfinite(s[i].center[0]) && std::isfinite(s[i].center[1]) &&
                                std::isfinite(s[i].center[2]) && std::isfinite(r[i]);
            if (!finite || r[i] > 64.f * med) always.push_back(i);
            else if (r[i] > 4.f * med) big.push_back(i);
            else small.push_back(i);
        }
    } else {
        for (uint32_t i = 0; i < n; ++i) always.push_back(i);
    }
    // clusters: the big ones, padded to a multiple of 4 (an empty slot never passes), then the
    // small ones; each group of 4 consecutive clusters gets a level-2 box
    std::vector<std::vector<uint32_t>> clusters;
    if (!big.empty()) split_clusters(s, big, clusters);
    while (clusters.size() % 4) clusters.emplace_back();
    if (!small.empty()) split_clusters(s, small, clusters);
    // clusters stay in the DFS order of the median-split tree: 4 consecutive clusters are a
    // depth-2 subtree, spatially tight, and become one level-2 box

    auto pad4 = [](uint32_t x) { return (x + 3u) & ~3u; };
    std::vector<float> geo;
    std::vector<uint32_t> sidx;
    auto push = [&](const std::vector<uint32_t> &ids) {
        const uint32_t base = static_cast<uint32_t>(sidx.size());
        for (uint32_t i : ids) {
            geo.insert(geo.end(), {s[i].center[0], s[i].center[1], s[i].center[2], s[i].radius * s[i].radius}); // raytracer.hxx:58
            sidx.push_back(i);
        }
        while (sidx.size() < base + pad4(static_cast<uint32_t>(ids.size()))) {
            geo.insert(geo.end(), {0.f, 0.f, 0.f, -INFINITY});  // never hits
            sidx.push_back(0xffffffffu);
        }
        return base;
    };
    blob_t b;
    push(always);
    b.always = always;
    b.n_always = static_cast<uint32_t>(always.size());  // tested with its exact count (padding after it)
    std::vector<float> crec;
    std::vector<float> boxes;  // per cluster lo/hi (6 floats), for the level-2 boxes
    for (const auto &c : clusters) {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t i : c)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], s[i].center[a] - std::fabs(s[i].radius));
                hi[a] = std::max(hi[a], s[i].center[a] + std::fabs(s[i].radius));
            }
        float C[3] = {0.f, 0.f, 0.f}, E[3] = {-1e30f, -1e30f, -1e30f};  // empty: no ray enters
        float kc = 0.f;
        if (!c.empty()) {
            for (int a = 0; a < 3; ++a) {
                C[a] = .5f * (lo[a] + hi[a]);
                E[a] = std::max(hi[a] - C[a], C[a] - lo[a]);
            }
            kc = kPadRel * (std::fabs(C[0]) + std::fabs(C[1]) + std::fabs(C[2]) + E[0] + E[1] + E[2]) + 1e-6f;
            b.clus_pad = std::max(b.clus_pad, kc);
        }
        boxes.insert(boxes.end(), {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
        const uint32_t start = push(c);
        const uint32_t cnt = pad4(static_cast<uint32_t>(c.size()));
        uint32_t packed = start | (cnt << 16);
        float pf;
        std::memcpy(&pf, &packed, 4);
        crec.insert(crec.end(), {C[0], C[1], C[2], E[0], E[1], E[2], kc, pf});
    }
    // 4 never-hitting entries after the last cluster: the transposed member tests read 16
    // member slots and mask the ones past the cluster's count
    for (int i = 0; i < 4; ++i) {
        geo.insert(geo.end(), {0.f, 0.f, 0.f, -INFINITY});
        sidx.push_back(0xffffffffu);
    }
    b.n_geo = static_cast<uint32_t>(sidx.size());
    b.n_clusters = static_cast<uint32_t>(clusters.size());
    b.n_clusters_real = b.n_clusters;
    // pad to a multiple of 4 clusters (grouped box tests) with boxes no ray enters:
    // negative extents make t_in > t_out whatever the ray
    while (b.n_clusters % 4) {
        uint32_t packed = static_cast<uint32_t>(sidx.size());  // count 0
        float pf;
        std::memcpy(&pf, &packed, 4);
        crec.insert(crec.end(), {0.f, 0.f, 0.f, -1e30f, -1e30f, -1e30f, 0.f, pf});
        ++b.n_clusters;
    }
    // layout in 16-byte units: geo | sidx (padded) | clusters
    b.data = geo;
    if (b.data.empty()) b.data.assign(4, 0.f);
    std::vector<uint32_t> sp = sidx;
    while (sp.size() % 4) sp.push_back(0xffffffffu);
    for (uint32_t v : sp) {
        float f;
        std::memcpy(&f, &v, 4);
        b.data.push_back(f);
    }
    b.clus_offset = static_cast<uint32_t>(b.data.size() / 4);
    b.data.insert(b.data.end(), crec.begin(), crec.end());
    // level 2: one box over every 4 consecutive clusters (padding clusters contribute nothing)
    b.supers_offset = static_cast<uint32_t>(b.data.size() / 4);
    for (uint32_t g = 0; g < b.n_clusters; g += 4) {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t c = g; c < std::min(g + 4, b.n_clusters_real); ++c)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], boxes[6 * c + a]);
                hi[a] = std::max(hi[a], boxes[6 * c + 3 + a]);
            }
        float C[3] = {0.f, 0.f, 0.f}, E[3] = {-1e30f, -1e30f, -1e30f};
        float kc = 0.f;
        if (lo[0] <= hi[0]) {
            for (int a = 0; a < 3; ++a) {
                C[a] = .5f * (lo[a] + hi[a]);
                E[a] = std::max(hi[a] - C[a], C[a] - lo[a]);
            }
            kc = kPadRel * (std::fabs(C[0]) + std::fabs(C[1]) + std::fabs(C[2]) + E[0] + E[1] + E[2]) + 1e-6f;
            b.clus_pad = std::max(b.clus_pad, kc);
        }
        uint32_t packed = g | (4u << 16);
        float pf;
        std::memcpy(&pf, &packed, 4);
        b.data.insert(b.data.end(), {C[0], C[1], C[2], E[0], E[1], E[2], kc, pf});
        ++b.n_supers;
    }
    // level 3: one box over every cluster (after the level-2 boxes)
    {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t c = 0; c < b.n_clusters_real; ++c)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], boxes[6 * c + a]);
                hi[a] = std::max(hi[a], boxes[6 * c + 3 + a]);
            }
        float C[3] = {0.f, 0.f, 0.f}, E[3] = {-1e30f, -1e30f, -1e30f};
        float kc = 0.f;
        if (lo[0] <= hi[0]) {
            for (int a = 0; a < 3; ++a) {
                C[a] = .5f * (lo[a] + hi[a]);
                E[a] = std::max(hi[a] - C[a], C[a] - lo[a]);
            }
            kc = kPadRel * (std::fabs(C[0]) + std::fabs(C[1]) + std::fabs(C[2]) + E[0] + E[1] + E[2]) + 1e-6f;
            b.clus_pad = std::max(b.clus_pad, kc);
        }
        uint32_t packed = 0;
        float pf;
        std::memcpy(&pf, &packed, 4);
        b.data.insert(b.data.end(), {C[0], C[1], C[2], E[0], E[1], E[2], kc, pf});
    }
    return b;
}

// The walk shortcut of dielectric spheres (rt_kernel.hip hint_candidate): a lane whose last hit
// was such a sphere S, whose next segment (0, 1.002 t] up to S's candidate t lies in the ball
// B(C, R_k) (R_k^2 = fl(fl(r r) kIsoR2Grow), the kernel's check of both ends), tests S's
// neighbours instead of walking the clusters. The neighbours N(S) are the clustered spheres
// T != S whose AABB, grown by the walk's own box pad for any origin in the ball, meets the ball;
// for every other T the segment misses every padded box the walk would test, and the walk's
// culling argument (such a T's candidate cannot beat t) holds sphere by sphere.
// So the minimum over S, N(S) and the always-tested spheres (the ground, tested anyway) is the
// walk's. R adds to R_k a margin for the float rounding of the kernel's check (a few ulp of
// |C| + r). Per sphere: kShortcut | (geo slot of neighbour 0, + 1) | (slot of neighbour 1, + 1)
// << 15 for spheres with at most two neighbours ("isolated": none), 0 otherwise.
// O(dielectric x clustered spheres) once per scene.
std::vector<uint32_t> shortcut_words(const rt_sphere *s, uint32_t n, const rt_material *m, const blob_t &b)
{
    std::vector<uint32_t> word(n, 0);
    if (b.n_clusters_real == 0) return word;  // no walk to skip
    // geo slot of each clustered sphere (blob layout: geo [n_geo] then sidx [n_geo])
    std::vector<uint32_t> slot(n, ~0u);
    for (uint32_t g = 0; g < b.n_geo; ++g) {
        uint32_t id;
        std::memcpy(&id, &b.data[4u * b.n_geo + g], 4);
        if (id < n && g >= b.n_always) slot[id] = g;
    }
    const bool slots_fit = b.n_geo < 0x7fffu;
    const char *e = std::getenv("RT_ISO_NB");  // RT_ISO_NB=0: isolated spheres only (A/B)
    const bool nb_off = e && e[0] == '0';
    std::vector<uint8_t> in_always(n, 0);
    for (uint32_t i : b.always) in_always[i] = 1;
    std::vector<uint32_t> others;
    size_t n_diel = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!in_always[i]) others.push_back(i);
        if (m[s[i].material].kind == RT_DIELECTRIC) ++n_diel;
    }
    if (static_cast<double>(n_diel) * static_cast<double>(others.size()) > 4e8) return word;  // leave huge scenes alone
    for (uint32_t S = 0; S < n && S < 0x7fffffffu; ++S) {
        if (m[s[S].material].kind != RT_DIELECTRIC) continue;
        const float r2 = s[S].radius * s[S].radius;  // the hint's geo entry, raytracer.hxx:58
        const float r2k = r2 * rt::kIsoR2Grow;        // the kernel's check radius, squared
        const double cx = s[S].center[0], cy = s[S].center[1], cz = s[S].center[2];
        if (!std::isfinite(cx) || !std::isfinite(cy) || !std::isfinite(cz) || !std::isfinite(r2k)) continue;
        const double rk = std::sqrt(static_cast<double>(r2k));
        const double c1 = std::fabs(cx) + std::fabs(cy) + std::fabs(cz);
        const double R = rk * (1.0 + 1e-5) + 1e-5 * (c1 + 2.0 * rk) + 1e-30;
        const double pad = 1e-3 * (c1 + 2.0 * R) + static_cast<double>(b.clus_pad) + 1e-6;
        const double C[3] = {cx, cy, cz};
        uint32_t nb[2], n_nb = 0;
        bool ok = true;
        for (uint32_t T : others) {
            if (T == S) continue;
            const double rt_ = std::fabs(static_cast<double>(s[T].radius));
            double d2 = 0.0;
            for (int a = 0; a < 3; ++a) {
                const double lo = s[T].center[a] - rt_ - pad, hi = s[T].center[a] + rt_ + pad;
                const double e = C[a] < lo ? lo - C[a] : (C[a] > hi ? C[a] - hi : 0.0);
                d2 += e * e;
            }
            if (!(d2 > R * R * (1.0 + 1e-9))) {
                if (n_nb == 2 || !slots_fit || slot[T] == ~0u) {
                    ok = false;
                    break;
                }
                nb[n_nb++] = slot[T];
            }
        }
        if (ok && n_nb && nb_off) ok = false;
        if (ok)
            word[S] = rt::kShortcut | (n_nb > 0 ? nb[0] + 1u : 0u) | (n_nb > 1 ? (nb[1] + 1u) << 15 : 0u);
    }
    return word;
}

uint32_t rows_of(const rt_params &p)
{
    if (p.num_rows) return p.num_rows;
    const uint32_t st = p.row_stride ? p.row_stride : 1;
    return p.row_offset >= p.height ? 0 : (p.height - p.row_offset + st - 1) / st;
}

int check_params(const rt_params *p)
{
    if (!p) return fail(RT_ERR_INVALID, "params: null");
    if (!p->width || !p->height || !p->spp) return fail(RT_ERR_INVALID, "params: width, height and spp must be > 0");
    // the kernel forms the pixel index y W + x in 32 bits (sample streams' keys)
    if (static_cast<uint64_t>(p->width) * p->height >= (1ull << 32))
        return fail(RT_ERR_INVALID, "params: width * height must be below 2^32");
    const uint32_t st = p->row_stride ? p->row_stride : 1;
    const uint32_t rows = rows_of(*p);
    if (rows && static_cast<uint64_t>(p->row_offset) + static_cast<uint64_t>(rows - 1) * st >= p->height)
        return fail(RT_ERR_INVALID, "params: rows exceed the image height");
    if (p->flags & ~(RT_FLAG_FULL_FRAME | RT_FLAG_FAST_MATH | RT_FLAG_SCALAR_SCENE | RT_FLAG_BRUTE_FORCE | RT_FLAG_CUDA_COMPAT |
                     RT_FLAG_WAVEFRONT))
        return fail(RT_ERR_INVALID, "params: unknown flag");
    return RT_OK;
}

rt::UDiv make_udiv(uint32_t d)
{
    rt::UDiv r{0, 0, 0};
    if (d <= 1) return r;  // d = 1: identity (t = 0, no shifts)
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    r.s1 = 1;
    r.s2 = l - 1;
    r.m = static_cast<uint32_t>(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    return r;
}

// Whether RN(a / b) == fma(fma(-q0, b, a), rb, q0) with rb = RN(1 / b), q0 = RN(a rb) for every
// a = m (m in [2^23, 2^24), i.e. every float mantissa). Powers of two scale every step exactly,
// so the identity then holds for every a >= 0 whose quotient and remainder stay normal: the
// kernel's x / width and x / height (x = 0, a pixel index, or a canonical draw >= 2^-32) use
// the two-FMA form when it holds. Checked once per divisor value (about 8 M host FMAs).
bool exact_by_reciprocal(float b)
{
    static std::mutex mu;
    static std::map<uint32_t, bool> cache;
    uint32_t key;
    std::memcpy(&key, &b, 4);
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    bool ok = std::isfinite(b) && b > 0.f && b >= 0x1p-60f && b <= 0x1p60f;
    const float rb = 1.f / b;
    for (uint32_t m = 1u << 23; ok && m < (1u << 24); ++m) {
        const float a = static_cast<float>(m);
        const float q0 = a * rb;
        const float q = std::fma(std::fma(-q0, b, a), rb, q0);
        ok = q == a / b;
    }
    std::lock_guard<std::mutex> g(mu);
    cache[key] = ok;
    return ok;
}

void fill_frame_consts(rt::KParams &k)
{
    rt::FrameConsts &f = k.fc;
    for (int c = 0; c < 3; ++c) { f.org[c] = k.org[c]; f.llc[c] = k.llc[c]; f.hor[c] = k.hor[c]; f.ver[c] = k.ver[c]; }
    f.lens = k.lens;
    f.fW = static_cast<float>(k.W);
    f.fH = static_cast<float>(k.H);
    f.corrected = k.corrected;
    f.W = k.W;
    f.spp = k.spp;
    f.inc_data_lo = static_cast<uint32_t>(k.inc_data);
    f.inc_data_hi = static_cast<uint32_t>(k.inc_data >> 32);
    f.inc_cam_lo = static_cast<uint32_t>(k.inc_cam);
    f.inc_cam_hi = static_cast<uint32_t>(k.inc_cam >> 32);
    f.row_offset = k.row_offset;
    f.row_stride = k.row_stride;
    f.tiled_rows = k.tiled_rows;
    f.tiles_x = k.tiles_x;
    f.tile_lw = k.tile_lw;
    f.n_pixels = k.n_pixels;
    f.sample_begin = k.sample_begin;
    f.div_W = make_udiv(k.W);
    f.div_tiles_x = make_udiv(k.tiles_x);
    f.div_n_pixels = make_udiv(k.n_pixels);
    f.rW = 1.f / f.fW;
    f.rH = 1.f / f.fH;
    f.div_fast = (exact_by_reciprocal(f.fW) ? 1u : 0u) | (exact_by_reciprocal(f.fH) ? 2u : 0u);
}

// A passing cluster requested by at most RT_TRANSPOSE_MAX lanes (default 16, at most 16; 0 =
// never) is tested transposed, (ray, member) pairs over the whole wave; same bits either way.
uint32_t transpose_max_env()
{
    const char *e = std::getenv("RT_TRANSPOSE_MAX");
    const unsigned long v = e && *e ? std::strtoul(e, nullptr, 10) : 16ul;
    return static_cast<uint32_t>(std::min<unsigned long>(v, 16ul));
}

// Short exact root forms (rt_kernel.hip RayDiv) when the scene and the camera lie within 2^19 of
// the origin; RT_FAST_ROOTS=0 keeps the IEEE sqrt/division sequences (A/B, tests); same bits.
bool fast_roots_env()
{
    const char *e = std::getenv("RT_FAST_ROOTS");
    return !(e && e[0] == '0');
}
bool camera_in_fast_range(const rt_camera &c)
{
    for (int i = 0; i < 3; ++i)
        for (float v : {c.origin[i], c.lower_left_corner[i], c.horizontal[i], c.vertical[i]})
            if (!(std::fabs(v) <= 0x1p19f)) return false;
    return std::fabs(c.lens_radius) <= 0x1p19f;
}

// RT_ROOT_BOX=0 disables the level-3 box gate (A/B); same bits either way.
uint32_t root_box_env()
{
    const char *e = std::getenv("RT_ROOT_BOX");
    return e && e[0] == '0' ? 0u : 1u;
}

// Deep-path split (render_kernel): paths that have traced RT_DEEP_SPLIT segments continue in a
// second launch of the same kernel that deals them densely (0 = no split). Same bits either way.
uint32_t deep_split_env()
{
    const char *e = std::getenv("RT_DEEP_SPLIT");
    return e && *e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : kDeepSplitDefault;
}
// deep queue of a pass: 8 regions of 1/1024 of its samples each (at least 512): 0.8% of the
// samples, where 0.2-0.3% reach the split depth on config 3; paths past a full region stay in the
// main launch. A pass of fewer than RT_DEEP_MIN_ITEMS samples (default 2^25) issued while no
// other render runs (a lone frame) is not split: its deep launch would be a serial tail of
// about max_depth - split iterations, which such a pass's own drain does not outweigh (config
// 3's 8-way row share alone: 1.28-1.30 ms split vs 1.03-1.10). Passes issued while others run
// (a frame stream) are split at any size: the unsplit drain costs issue (the 8-way share ran
// 42% more VALU instructions per sample than the full frame) and the deep launches run beside
// the other frames (8-way share, 7 streams: 0.50-0.51 ms per frame vs 0.58-0.59 unsplit).
uint32_t deep_region_cap(uint32_t n_items)
{
    const char *e = std::getenv("RT_DEEP_REGION_DIV");
    const unsigned long div = e && *e ? std::max(1ul, std::strtoul(e, nullptr, 10)) : 1024ul;
    return std::max<uint32_t>(512u, static_cast<uint32_t>(n_items / div));
}
// The deep launch's waves take the highest issue priority (RT_DEEP_PRIO=0 turns it off, A/B):
// its paths are chains of ~56 dependent iterations, and beside other renders' waves each
// iteration waits for the SIMD's other waves. Config 3's 8-way row share, split, 7 streams:
// 0.513-0.515 ms vs 0.569-0.571 (profiles/r03/ab/deep_prio.txt); the full frame alike.
uint32_t deep_prio_env()
{
    const char *e = std::getenv("RT_DEEP_PRIO");
    return e && e[0] == '0' ? 0u : 1u;
}

// RT_ISO=0 turns off the isolated-sphere shortcut of the cluster walk (rt_kernel.hip
// hint_candidate; A/B and tests; default on)
uint32_t iso_env()
{
    const char *e = std::getenv("RT_ISO");
    return e && e[0] == '0' ? 0u : 1u;
}

// RT_DEEP_ROOT_BOX=1 keeps the level-3 box gate in the deep launch (A/B; default off)
bool deep_root_box_env()
{
    const char *e = std::getenv("RT_DEEP_ROOT_BOX");
    return e && e[0] == '1';
}
// a nonzero key of the camera basis and the depth limit (FNV-1a over their bytes)
unsigned long long camera_key(const rt_camera &c, uint32_t max_depth)
{
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) {
        for (size_t i = 0; i < n; ++i) h = (h ^ static_cast<const unsigned char *>(p)[i]) * 1099511628211ull;
    };
    mix(&c, sizeof(c));
    mix(&max_depth, sizeof(max_depth));
    return h ? h : 1ull;
}
uint64_t deep_min_items_env()
{
    const char *e = std::getenv("RT_DEEP_MIN_ITEMS");
    return e && *e ? std::strtoull(e, nullptr, 10) : (1ull << 25);
}

} // namespace

struct rt_scene;
namespace {

// RT_FLAG_CUDA_COMPAT: the reference's CUDA variant semantics (compat_kernel), on the caller
// stream, spheres read from the index-ordered shading records of the brute-force blob.
int render_compat(rt_scene *sc, const rt_camera *camera, const rt_params &P, float *d_rgb, hipStream_t st,
                  uint64_t *d_segments);

// Render passes in flight: RT_PIPELINE=0 (or 1) runs the render kernels on the caller stream;
// 2..kMaxBufs rotate that many internal streams. Default: one stream fewer than the process's
// hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4; the caller's stream takes one), 2..4.
// The max-depth paths give every launch a drain of ~64 iterations whatever its size; with 3
// streams (and partial grids, grid_wg_per_cu) two other renders fill the machine while one
// drains. Measured on config 3 (frame stream): 3.81-3.87 ms/frame with 3 streams vs 3.90-3.93
// with 2; an 8-way row share (14.7 M samples) 0.63-0.64 vs 0.68; 4 streams on 8 hardware
// queues: 3.83-3.84 and 0.61. More streams than hardware queues share queues and serialise.
uint32_t pipeline_env()
{
    const char *e = std::getenv("RT_PIPELINE");
    if (!e || !*e) {
        const char *q = std::getenv("GPU_MAX_HW_QUEUES");
        const unsigned long hw = q && *q ? std::strtoul(q, nullptr, 10) : 4ul;
        // at most 7: with row shares split (passes in flight) 7 streams beat 4 (config 3's 8-way
        // share 0.50 vs 0.58 ms, 4-way 0.88 vs 0.95; the full frame 2.99-3.04 vs 3.06-3.08) and
        // 8 (on 12 hardware queues) is slower again (profiles/r03/ab); each stream holds two
        // slot workspaces
        return static_cast<uint32_t>(std::clamp<unsigned long>(hw > 1 ? hw - 1 : 1, 2, 7));
    }
    const unsigned long v = std::strtoul(e, nullptr, 10);
    return v <= 1 ? 1u : static_cast<uint32_t>(std::min<unsigned long>(v, kMaxBufs));
}

// Workspaces per internal stream (RT_WS_PER_STREAM, 1..2; default 2). Pass p renders on stream
// p % streams into workspace p % (streams x this): with 2, the render that next takes a stream
// waits only for that stream's previous render (stream order), not for the accumulation of
// the pass that last used its workspace, which runs on the caller stream and, beside the
// running renders, waits for free CU slots.
uint32_t ws_per_stream_env()
{
    const char *e = std::getenv("RT_WS_PER_STREAM");
    if (!e || !*e) return 2u;
    const unsigned long v = std::strtoul(e, nullptr, 10);
    return v <= 1 ? 1u : static_cast<uint32_t>(std::min<unsigned long>(v, kMaxWs / kMaxBufs));
}

// RT_DEBUG_STATS=1 selects the diagnostic instantiation (same bits, extra counters).
bool debug_stats()
{
    const char *e = std::getenv("RT_DEBUG_STATS");
    return e && e[0] == '1';
}

// RT_SHADE_LDS=0/1 forces the shading records out of / into LDS (-1 = automatic).
int shade_lds_env()
{
    const char *e = std::getenv("RT_SHADE_LDS");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
}

// the render kernels' static LDS (per-wave transposed-test records 4 x 640 B, per-lane pending
// normal 256 x 16 B, hint index and shortcut word 2 x 256 x 4 B: 8704 B), with a margin
constexpr size_t kRenderStaticLds = 12u << 10;

// RT_DEEP_SHADE_LDS=0 keeps the deep launch's shading records in global memory (A/B; default 1)
bool deep_shade_lds_env()
{
    const char *e = std::getenv("RT_DEEP_SHADE_LDS");
    return !(e && e[0] == '0');
}

// RT_VERBOSE=1 prints each launch's plan (variant, LDS bytes, occupancy, grid, items) to stderr.
bool verbose()
{
    const char *e = std::getenv("RT_VERBOSE");
    return e && e[0] == '1';
}

int ensure(void **ptr, size_t *have, size_t want)
{
    if (*have >= want && *ptr) return RT_OK;
    if (*ptr) {
        RT_HIP(hipDeviceSynchronize());
        RT_HIP(hipFree(*ptr));
        *ptr = nullptr;
        *have = 0;
    }
    RT_HIP(hipMalloc(ptr, std::max<size_t>(want, 256)));
    *have = want;
    return RT_OK;
}

} // namespace

extern "C" {

int rt_scene_simple(rt_sphere *spheres, uint32_t sphere_cap, uint32_t *n_spheres, rt_material *materials,
                    uint32_t material_cap, uint32_t *n_materials)
{
    scene_builder b;
    b.simple();
    return b.emit(spheres, sphere_cap, n_spheres, materials, material_cap, n_materials);
}

int rt_scene_cuda(rt_sphere *spheres, uint32_t sphere_cap, uint32_t *n_spheres, rt_material *materials,
                  uint32_t material_cap, uint32_t *n_materials)
{
    scene_builder b;
    b.cuda_variant();
    return b.emit(spheres, sphere_cap, n_spheres, materials, material_cap, n_materials);
}

int rt_scene_huge(uint32_t seed, rt_sphere *spheres, uint32_t sphere_cap, uint32_t *n_spheres,
                  rt_material *materials, uint32_t material_cap, uint32_t *n_materials)
{
    scene_builder b;
    b.huge(seed);
    return b.emit(spheres, sphere_cap, n_spheres, materials, material_cap, n_materials);
}

int rt_scene_destroy(rt_scene *sc)
{
    if (!sc) return RT_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(sc->device);
    for (auto e : sc->ev_begin) (void)hipEventDestroy(e);
    for (auto e : sc->ev_end) (void)hipEventDestroy(e);
    for (uint32_t b = 0; b < kMaxBufs; ++b) {
        if (sc->xs[b]) (void)hipStreamSynchronize(sc->xs[b]);
        if (sc->xs[b]) (void)hipStreamDestroy(sc->xs[b]);
    }
    for (uint32_t b = 0; b < kMaxWs; ++b) {
        if (sc->ev_done[b]) (void)hipEventDestroy(sc->ev_done[b]);
        if (sc->ev_free[b]) (void)hipEventDestroy(sc->ev_free[b]);
        if (sc->ev_main[b]) (void)hipEventDestroy(sc->ev_main[b]);
    }
    if (sc->ev_tail) (void)hipEventDestroy(sc->ev_tail);
    for (void *p : {(void *)sc->blob[0], (void *)sc->blob[1], (void *)sc->dbg, (void *)sc->acc, (void *)sc->queue_ctr, sc->wq})
        if (p) (void)hipFree(p);
    for (float *p : sc->slots)
        if (p) (void)hipFree(p);
    for (void *p : sc->deep)
        if (p) (void)hipFree(p);
    if (sc->deep_over) (void)hipHostFree(sc->deep_over);
    (void)hipSetDevice(prev);
    delete sc;
    return RT_OK;
}

int rt_scene_create(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials,
                    uint32_t n_materials, int device, rt_scene **out)
{
    if (!out || (n_spheres && !spheres) || !materials || !n_materials)
        return fail(RT_ERR_INVALID, "rt_scene_create: null argument or no materials");
    *out = nullptr;
    for (uint32_t i = 0; i < n_spheres; ++i)
        if (spheres[i].material >= n_materials)
            return fail(RT_ERR_INVALID, "rt_scene_create: sphere " + std::to_string(i) + " has material index " +
                                            std::to_string(spheres[i].material) + " >= " + std::to_string(n_materials));
    for (uint32_t i = 0; i < n_materials; ++i)
        if (materials[i].kind > RT_DIELECTRIC)
            return fail(RT_ERR_INVALID, "rt_scene_create: material " + std::to_string(i) + " has unknown kind");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_ERR_DEVICE, "rt_scene_create: no HIP device");
    if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID, "rt_scene_create: bad device index");
    RT_HIP(hipSetDevice(device));

    std::vector<float> hit(static_cast<size_t>(std::max(n_spheres, 1u)) * 12, 0.f);
    for (uint32_t i = 0; i < n_spheres; ++i) {
        const rt_sphere &sp = spheres[i];
        const rt_material &mt = materials[sp.material];
        float *h = hit.data() + 12 * static_cast<size_t>(i);
        h[0] = sp.center[0]; h[1] = sp.center[1]; h[2] = sp.center[2]; h[3] = sp.radius;
        h[4] = mt.albedo[0]; h[5] = mt.albedo[1]; h[6] = mt.albedo[2]; h[7] = mt.param;
        std::memcpy(h + 8, &mt.kind, 4);
    }
    blob_t blobs[2] = {build_blob(spheres, n_spheres, false), build_blob(spheres, n_spheres, true)};
    const std::vector<uint32_t> shortcut = shortcut_words(spheres, n_spheres, materials, blobs[1]);
    // shading records join each blob (so they sit in LDS next to the geometry): per original
    // sphere index {c, r}, {albedo, param}, then the material kinds as bytes, 16-B padded
    for (blob_t &b : blobs) {
        b.shade_offset = static_cast<uint32_t>(b.data.size() / 4);
        for (uint32_t i = 0; i < n_spheres; ++i) b.data.insert(b.data.end(), hit.data() + 12 * static_cast<size_t>(i), hit.data() + 12 * static_cast<size_t>(i) + 8);
        std::vector<uint8_t> kinds((n_spheres + 15u) / 16u * 16u, 0);
        for (uint32_t i = 0; i < n_spheres; ++i) kinds[i] = static_cast<uint8_t>(materials[spheres[i].material].kind);
        const size_t at = b.data.size();
        b.data.resize(at + kinds.size() / 4);
        std::memcpy(b.data.data() + at, kinds.data(), kinds.size());
        // dielectric constants per sphere index (raytracer.hxx:166-174 and the Schlick ratio
        // :47): {1 / ior, (1 - ior) / (1 + ior), (1 - 1/ior) / (1 + 1/ior), shortcut}, the same
        // binary32 operations the kernel would run (this file is built with -ffp-contract=off);
        // and the sphere's walk-shortcut word (shortcut_words; as raw bits)
        for (uint32_t i = 0; i < n_spheres; ++i) {
            const rt_material &mt = materials[spheres[i].material];
            float dc[4] = {0.f, 0.f, 0.f, 0.f};
            if (mt.kind == RT_DIELECTRIC) {
                const float ior = mt.param, inv = 1.f / ior;
                dc[0] = inv;
                dc[1] = (1.f - ior) / (1.f + ior);
                dc[2] = (1.f - inv) / (1.f + inv);
                std::memcpy(&dc[3], &shortcut[i], 4);
            }
            b.data.insert(b.data.end(), dc, dc + 4);
        }
    }
    rt_scene *sc = new rt_scene();
    for (auto &r : sc->occ) for (auto &x : r) x[0] = x[1] = -1;
    sc->in_fast_range = true;
    for (uint32_t i = 0; i < n_spheres; ++i) {
        for (float v : {spheres[i].center[0], spheres[i].center[1], spheres[i].center[2], spheres[i].radius})
            if (!(std::fabs(v) <= 0x1p19f)) sc->in_fast_range = false;
        // the hit normal's short division by r (rt_kernel.hip div3_short) needs |r| >= 2^-40
        if (!(std::fabs(spheres[i].radius) >= 0x1p-40f)) sc->in_fast_range = false;
    }
    sc->device = device;
    sc->n_spheres = n_spheres;
    sc->n_materials = n_materials;
    auto up = [&](void **dst, const void *src, size_t bytes) -> int {
        RT_HIP(hipMalloc(dst, bytes));
        RT_HIP(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
        return RT_OK;
    };
    int rc = RT_OK;
    for (int b = 0; b < 2 && rc == RT_OK; ++b) {
        rc = up((void **)&sc->blob[b], blobs[b].data.data(), blobs[b].data.size() * 4);
        sc->blob_units[b] = static_cast<uint32_t>(blobs[b].data.size() / 4);
        sc->n_geo[b] = blobs[b].n_geo;
        sc->n_always[b] = blobs[b].n_always;
        sc->n_clusters[b] = blobs[b].n_clusters;
        sc->clus_offset[b] = blobs[b].clus_offset;
        sc->clus_pad[b] = blobs[b].clus_pad;
        sc->n_supers[b] = blobs[b].n_supers;
        sc->supers_offset[b] = blobs[b].supers_offset;
        sc->shade_offset[b] = blobs[b].shade_offset;
    }
    if (rc == RT_OK) {
        hipError_t e = hipMalloc((void **)&sc->queue_ctr, kCtrWords * sizeof(uint32_t));
        if (e != hipSuccess) rc = fail(RT_ERR_DEVICE, std::string("hipMalloc: ") + hipGetErrorString(e));
        if (rc == RT_OK &&
            (hipHostMalloc((void **)&sc->deep_over, kMaxWs * sizeof(unsigned long long), hipHostMallocMapped) != hipSuccess ||
             hipHostGetDevicePointer((void **)&sc->deep_over_dev, sc->deep_over, 0) != hipSuccess))
            rc = fail(RT_ERR_DEVICE, "rt_scene_create: pinned host allocation failed");
        if (rc == RT_OK) std::memset(sc->deep_over, 0, kMaxWs * sizeof(unsigned long long));
        for (uint32_t b = 0; b < kMaxWs && rc == RT_OK; ++b) {
            if ((b < kMaxBufs && hipStreamCreateWithFlags(&sc->xs[b], hipStreamNonBlocking) != hipSuccess) ||
                hipEventCreateWithFlags(&sc->ev_done[b], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&sc->ev_free[b], hipEventDisableTiming) != hipSuccess)
                rc = fail(RT_ERR_DEVICE, "rt_scene_create: stream/event creation failed");
        }
        if (rc == RT_OK && hipEventCreateWithFlags(&sc->ev_tail, hipEventDisableTiming) != hipSuccess)
            rc = fail(RT_ERR_DEVICE, "rt_scene_create: event creation failed");
    }
    if (rc == RT_OK) {
        hipDeviceProp_t prop;
        hipError_t e = hipGetDeviceProperties(&prop, device);
        if (e != hipSuccess) rc = fail(RT_ERR_DEVICE, std::string("hipGetDeviceProperties: ") + hipGetErrorString(e));
        else {
            sc->cu_count = prop.multiProcessorCount;
            sc->max_lds = prop.sharedMemPerBlock;
        }
    }
    for (uint32_t i = 0; rc == RT_OK && i < rt_scene::kRing; ++i) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
            if (a) (void)hipEventDestroy(a);
            rc = fail(RT_ERR_DEVICE, "hipEventCreate failed");
            break;
        }
        sc->ev_begin.push_back(a);
        sc->ev_end.push_back(b);
    }
    if (rc != RT_OK) {
        rt_scene_destroy(sc);
        return rc;
    }
    *out = sc;
    return RT_OK;
}

namespace {
// Calls on one scene may come on different caller streams: order a call after everything the
// previous call enqueued on its stream (the accumulation buffer and counters are
// per scene), then remember this call's stream and its last work.
int stream_enter(rt_scene *sc, hipStream_t st)
{
    if (sc->tail_valid && st != sc->last_stream) RT_HIP(hipStreamWaitEvent(st, sc->ev_tail, 0));
    return RT_OK;
}
int stream_leave(rt_scene *sc, hipStream_t st)
{
    RT_HIP(hipEventRecord(sc->ev_tail, st));
    sc->last_stream = st;
    sc->tail_valid = true;
    return RT_OK;
}
int render_device_impl(rt_scene *sc, const rt_camera *camera, const rt_params &P, float *d_rgb, hipStream_t st,
                       uint64_t *d_segments);
} // namespace

int rt_render_device(rt_scene *sc, const rt_camera *camera, const rt_params *params, float *d_rgb, void *stream,
                     uint64_t *d_segments)
{
    if (!sc || !camera || !d_rgb) return fail(RT_ERR_INVALID, "rt_render_device: null argument");
    if (int rc = check_params(params); rc != RT_OK) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    RT_HIP(hipSetDevice(sc->device));
    if (int rc = stream_enter(sc, st); rc != RT_OK) return rc;
    const int rc = (params->flags & RT_FLAG_CUDA_COMPAT) ? render_compat(sc, camera, *params, d_rgb, st, d_segments)
                                                         : render_device_impl(sc, camera, *params, d_rgb, st, d_segments);
    if (rc != RT_OK) return rc;
    return stream_leave(sc, st);
}

namespace {
int render_device_impl(rt_scene *sc, const rt_camera *camera, const rt_params &P, float *d_rgb, hipStream_t st,
                       uint64_t *d_segments)
{
    rt::KParams k{};
    for (int c = 0; c < 3; ++c) {
        k.org[c] = camera->origin[c];
        k.llc[c] = camera->lower_left_corner[c];
        k.hor[c] = camera->horizontal[c];
        k.ver[c] = camera->vertical[c];
    }
    k.lens = camera->lens_radius;
    k.corrected = camera->mode == RT_CAMERA_CORRECTED;
    k.W = P.width;
    k.H = P.height;
    k.spp = P.spp;
    k.max_depth = P.max_depth;
    k.row_offset = P.row_offset;
    k.row_stride = P.row_stride ? P.row_stride : 1;
    k.num_rows = rows_of(P);
    k.full_frame = (P.flags & RT_FLAG_FULL_FRAME) ? 1u : 0u;
    k.inc_data = ((2ull * P.seed) << 1u) | 1ull;
    k.inc_cam = ((2ull * P.seed + 1ull) << 1u) | 1ull;
    const uint64_t n_pixels = static_cast<uint64_t>(P.width) * k.num_rows;
    if (n_pixels == 0) return RT_OK;
    if (n_pixels >= (1ull << 31)) return fail(RT_ERR_INVALID, "rt_render_device: more than 2^31 pixels in one call");
    k.n_pixels = static_cast<uint32_t>(n_pixels);
    // 64-pixel tiles (one wave's lanes for one sample), 2^lw wide and 64/2^lw rows tall
    k.tile_lw = tile_lw_for(P.width, k.row_stride);
    const uint32_t tw = 1u << k.tile_lw, th = 64u >> k.tile_lw;
    const bool tiled = (P.width % tw) == 0u;
    k.tiles_x = tiled ? P.width / tw : 1u;
    k.tiled_rows = tiled ? (k.num_rows / th) * th : 0u;
    k.n_spheres = sc->n_spheres;
    k.n_materials = sc->n_materials;


    // Variant: exact (bit-exact) or fast (tolerance); clustered culling unless brute force is
    // asked for; the scalar-cache A/B variant is brute force only. Each needs its blob in LDS.
    int variant = (P.flags & RT_FLAG_FAST_MATH) ? rt::V_FAST_LDS : rt::V_EXACT_LDS;
    bool cull = !(P.flags & RT_FLAG_BRUTE_FORCE) && sc->n_clusters[1] > 0;
    const bool wave = (P.flags & RT_FLAG_WAVEFRONT) != 0u;
    if (wave && (P.flags & (RT_FLAG_FAST_MATH | RT_FLAG_SCALAR_SCENE)))
        return fail(RT_ERR_UNSUPPORTED, "rt_render_device: the wavefront variant is the exact kernel only");
    if (P.flags & RT_FLAG_SCALAR_SCENE) { variant = rt::V_EXACT_SCALAR; cull = false; }
    if (variant != rt::V_EXACT_SCALAR && static_cast<size_t>(sc->shade_offset[cull]) * 16u > sc->max_lds) {
        if (variant == rt::V_FAST_LDS || cull) return fail(RT_ERR_UNSUPPORTED, "rt_render_device: scene too large for LDS");
        variant = rt::V_EXACT_SCALAR;
    }
    if (wave && variant != rt::V_EXACT_LDS)
        return fail(RT_ERR_UNSUPPORTED, "rt_render_device: the wavefront variant needs the scene in LDS");
    if (variant == rt::V_EXACT_LDS && debug_stats() && !wave) {
        variant = rt::V_STATS_LDS;
        if (!sc->dbg) {
            RT_HIP(hipMalloc((void **)&sc->dbg, rt::kDbgWords * sizeof(unsigned long long)));
            RT_HIP(hipMemset(sc->dbg, 0, rt::kDbgWords * sizeof(unsigned long long)));
        }
        k.dbg = sc->dbg;
    }
    const int b = cull ? 1 : 0;
    const int cull_mode = cull ? 7 : 0;
    k.blob = reinterpret_cast<const float4 *>(sc->blob[b]);
    k.blob_units = sc->blob_units[b];
    k.n_geo = sc->n_geo[b];
    k.n_always = sc->n_always[b];
    k.n_clusters = sc->n_clusters[b];
    k.clus_offset = sc->clus_offset[b];
    k.clus_pad = sc->clus_pad[b];
    k.n_supers = sc->n_supers[b];
    k.supers_offset = sc->supers_offset[b];
    k.use_root = root_box_env();
    k.iso = iso_env();
    k.transpose_max = transpose_max_env();
    k.fast_roots = sc->in_fast_range && camera_in_fast_range(*camera) && fast_roots_env() ? 1u : 0u;
    k.shade_offset = sc->shade_offset[b];
    // the shading records (the blob's tail) join the geometry in LDS unless that costs
    // workgroups per CU; RT_SHADE_LDS=0/1 forces the choice for A/B
    auto occ_for = [&](int in_lds, int *out) -> int {
        int &o = sc->occ[variant][cull ? 1 : 0][in_lds];
        if (o < 0) {
            const size_t bytes = variant == rt::V_EXACT_SCALAR ? 0 : static_cast<size_t>(in_lds ? k.blob_units : k.shade_offset) * 16u;
            RT_HIP(rt::occupancy_render(variant, cull_mode, &o, bytes));
            o = std::max(o, 1);
        }
        *out = o;
        return RT_OK;
    };
    int occ_geo = 0, occ_all = 0;
    if (int rc = occ_for(0, &occ_geo); rc) return rc;
    if (int rc = occ_for(1, &occ_all); rc) return rc;
    const int force = shade_lds_env();
    k.shade_lds = variant != rt::V_EXACT_SCALAR && static_cast<size_t>(k.blob_units) * 16u <= sc->max_lds &&
                  (force >= 0 ? force == 1 : occ_all >= occ_geo);
    k.lds_units = variant == rt::V_EXACT_SCALAR ? 0u : (k.shade_lds ? k.blob_units : k.shade_offset);
    const size_t lds = static_cast<size_t>(k.lds_units) * 16u;
    const int occ = k.shade_lds ? occ_all : occ_geo;

    // pass planning: the slot workspace of one pass (12 B per sample and pixel) stays under
    // the budget; passes hold a multiple of 4 samples so no reduce block straddles two
    const uint64_t per_sample = n_pixels * 12ull;
    uint64_t spp_pass = std::min<uint64_t>(P.spp, slot_budget() / per_sample);
    spp_pass = std::min<uint64_t>(spp_pass, ((1ull << 31) - 8192) / n_pixels);  // items fit 31 bits
    if (spp_pass < P.spp) spp_pass &= ~3ull;
    if (spp_pass == 0) spp_pass = 4;
    if (n_pixels * std::min<uint64_t>(spp_pass, P.spp) >= (1ull << 31) - 8192)
        return fail(RT_ERR_INVALID, "rt_render_device: too many pixels in one call");
    // frames in flight: render pass p runs on internal stream xs[p % bufs] with workspace
    // w = p % n_ws, ordered after that stream's previous render and after the caller-stream
    // work that last read workspace w (the accumulation of pass p - n_ws); render kernels
    // touch no caller memory, so the caller stream sees the same results in the same order.
    // RT_PIPELINE=0: everything on the caller stream.
    // deep-path split, unless a pass with this camera (and depth limit) has overflowed the deep
    // queue on this scene: paths that long are common there (the corrected camera: 8.4% of the
    // samples pass 8 segments, 59% of the segments), and a partial split only adds a tail
    for (uint32_t w = 0; w < kMaxWs; ++w) {
        // take-and-clear in one atomic step: a report the device writes meanwhile is kept
        const unsigned long long v = __atomic_exchange_n(sc->deep_over + w, 0ull, __ATOMIC_ACQ_REL);
        if (!v) continue;
        auto it = std::find_if(sc->deep_off.begin(), sc->deep_off.end(), [&](const auto &e) { return e.first == v; });
        if (it != sc->deep_off.end()) sc->deep_off.erase(it);
        else if (sc->deep_off.size() >= rt_scene::kDeepOffKeys) sc->deep_off.erase(sc->deep_off.begin());
        sc->deep_off.emplace_back(v, sc->calls);  // most recent last
    }
    // reports expire: a camera is tried split again kDeepOffCalls calls after its last overflow
    sc->deep_off.erase(std::remove_if(sc->deep_off.begin(), sc->deep_off.end(),
                                      [&](const auto &e) { return sc->calls - e.second > rt_scene::kDeepOffCalls; }),
                       sc->deep_off.end());
    const unsigned long long deep_key = camera_key(*camera, P.max_depth);
    const bool deep_off = std::find_if(sc->deep_off.begin(), sc->deep_off.end(),
                                       [&](const auto &e) { return e.first == deep_key; }) != sc->deep_off.end();
    const uint32_t deep_split = deep_off ? 0u : deep_split_env();
    const uint64_t deep_min_items = deep_min_items_env();
    const uint32_t bufs = wave ? 1u : pipeline_env();  // the wavefront variant: caller stream only
    const bool pipe = bufs > 1;
    const uint32_t n_ws = pipe ? bufs * ws_per_stream_env() : 1u;
    if (spp_pass < P.spp)
        if (int rc = ensure((void **)&sc->acc, &sc->acc_bytes, per_sample); rc) return rc;
    for (uint32_t w = 0; w < n_ws; ++w)
        if (int rc = ensure((void **)&sc->slots[w], &sc->slots_bytes[w], per_sample * std::min<uint64_t>(spp_pass, P.spp)); rc)
            return rc;
    k.chunk_items = chunk_items();
    // wavefront variant: two ray queues of cap rays (52 B each) and their counters
    uint32_t wcap = 0;
    rt::RayQueue wqa{}, wqb{};
    int wgrid = 0;
    if (wave) {
        wcap = static_cast<uint32_t>(std::min<uint64_t>(n_pixels * std::min<uint64_t>(spp_pass, P.spp), wave_queue_env()));
        const size_t qbytes = static_cast<size_t>(wcap) * 52u;
        if (int rc = ensure(&sc->wq, &sc->wq_bytes, 2 * qbytes + 512); rc) return rc;
        auto carve = [&](char *base, rt::RayQueue &q) {
            q.f = reinterpret_cast<float *>(base);
            q.rng = reinterpret_cast<uint64_t *>(base + static_cast<size_t>(wcap) * 36u);
            q.item = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(wcap) * 44u);
            q.depth = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(wcap) * 48u);
        };
        char *w0 = static_cast<char *>(sc->wq);
        carve(w0, wqa);
        carve(w0 + qbytes, wqb);
        wqa.count = reinterpret_cast<uint32_t *>(w0 + 2 * qbytes);
        wqb.count = reinterpret_cast<uint32_t *>(w0 + 2 * qbytes + 256);
        int &ow = sc->occ_wave[cull ? 1 : 0];
        if (ow < 0) {
            RT_HIP(rt::occupancy_wave_bounce(cull_mode, &ow, lds));
            ow = std::max(ow, 1);
        }
        wgrid = ow * sc->cu_count;
    }

    const uint32_t ring = static_cast<uint32_t>(sc->calls % rt_scene::kRing);
    ++sc->calls;
    const uint32_t full_blocks_end = P.spp & ~3u;  // samples [0, full_blocks_end) form blocks of 4
    for (uint32_t s0 = 0; s0 < P.spp; s0 += static_cast<uint32_t>(spp_pass)) {
        const uint32_t s1 = static_cast<uint32_t>(std::min<uint64_t>(P.spp, s0 + spp_pass));
        // every pass takes the next workspace and stream: pass p + 1's render overlaps pass
        // p's drain and accumulation, within a frame and across frames
        const uint32_t wb = pipe ? sc->next_buf % n_ws : 0u;
        sc->next_buf = wb + 1u;
        hipStream_t xst = pipe ? sc->xs[wb % bufs] : st;
        // another render still running? (then this one takes a partial grid, grid_wg_per_cu)
        const bool in_flight = pipe && sc->last_ws >= 0 && hipEventQuery(sc->ev_done[sc->last_ws]) == hipErrorNotReady;
        k.slots = sc->slots[wb];
        k.queue_ctr = sc->queue_ctr + wb * 8u * rt::kQueueStride;
        unsigned long long *seg_b = reinterpret_cast<unsigned long long *>(sc->queue_ctr + kSegWords) + 4u * wb;
        k.segments = d_segments ? (pipe ? seg_b : reinterpret_cast<unsigned long long *>(d_segments)) : nullptr;
        if (pipe && sc->free_valid[wb]) RT_HIP(hipStreamWaitEvent(xst, sc->ev_free[wb], 0));
        if (sc->ctr_dirty[wb]) {
            RT_HIP(hipMemsetAsync(k.queue_ctr, 0, 8 * rt::kQueueStride * sizeof(uint32_t), xst));
            RT_HIP(hipMemsetAsync(seg_b, 0, 3 * sizeof(unsigned long long), xst));
        }
        sc->ctr_dirty[wb] = true;
        if (s0 == 0) RT_HIP(hipEventRecord(sc->ev_begin[ring], xst));
        k.sample_begin = s0;
        k.sample_end = s1;
        fill_frame_consts(k);
        k.n_items = static_cast<uint32_t>(n_pixels * (s1 - s0));
        {   // the last tail_pct % of the items go out in 64-item chunks (even end-of-launch drain)
            const uint64_t tail = static_cast<uint64_t>(k.n_items) * tail_pct() / 100u;
            k.n_big_chunks = static_cast<uint32_t>((k.n_items - tail) / k.chunk_items);
            const uint32_t rest = k.n_items - k.n_big_chunks * k.chunk_items;
            k.n_chunks = k.n_big_chunks + (rest + 63u) / 64u;
        }
        const uint32_t grid = static_cast<uint32_t>(
            std::max<uint64_t>(1, std::min<uint64_t>(static_cast<uint64_t>(grid_wg_per_cu(occ, in_flight, bufs, k.n_items)) * sc->cu_count, (k.n_items + 255u) / 256u)));
        k.n_blocks = (k.n_items + 63u) / 64u;
        k.guided_l2b = guided_l2b(grid * 4u, in_flight);
        // deep-path split: this workspace's deep queue (its counters in the queue-counter block)
        k.deep_depth = 0;
        k.deep_mode = 0;
        bool two_part = false;
        // culled scenes only: with a handful of spheres (the simple scene, brute force) a deep
        // segment is cheap and the deep launch's overhead outweighs the drain it saves
        // (config 2: 0.98-1.00 vs 0.98-0.99 ms per frame)
        if (deep_split && !wave && cull_mode == 7 && deep_split < P.max_depth && (k.n_items >= deep_min_items || in_flight)) {
            const uint32_t rcap = deep_region_cap(k.n_items), cap = 8u * rcap;
            const size_t px_bytes = (n_pixels + 255u) & ~static_cast<size_t>(255u);
            void *had = sc->deep[wb];
            if (int rc = ensure(&sc->deep[wb], &sc->deep_bytes[wb], px_bytes + static_cast<size_t>(cap) * 52u); rc) return rc;
            if (sc->deep[wb] != had) sc->deep_clean[wb] = 0;  // new memory
            if (sc->deep_clean[wb] < px_bytes) {  // flags over bytes a queue may have used
                RT_HIP(hipMemsetAsync(sc->deep[wb], 0, px_bytes, xst));
                sc->deep_clean[wb] = px_bytes;
            }
            char *base = static_cast<char *>(sc->deep[wb]);
            k.deep.px = reinterpret_cast<uint8_t *>(base);
            base += px_bytes;
            k.deep.f = reinterpret_cast<float *>(base);
            k.deep.rng = reinterpret_cast<uint64_t *>(base + static_cast<size_t>(cap) * 36u);
            k.deep.slot = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(cap) * 44u);
            k.deep.hid = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(cap) * 48u);
            k.deep.ctr = k.queue_ctr;
            k.deep.rcap = rcap;
            k.deep_depth = deep_split;
            two_part = pipe && !in_flight;
        }
        if (verbose())
            std::fprintf(stderr, "[rt] variant=%d cull=%d shade_lds=%u lds=%zu B occ=%d WG/CU cus=%d grid=%u items=%u samples=[%u,%u) %s%u\n",
                         variant, cull_mode, k.shade_lds, lds, occ, sc->cu_count, grid, k.n_items, s0, s1,
                         k.guided_l2b < 0.f ? "guided log2(beta)*1e6=" : "chunk=",
                         k.guided_l2b < 0.f ? static_cast<uint32_t>(-k.guided_l2b * 1e6f) : k.chunk_items);
        if (wave) {
            // items in chunks of wcap: one generation launch, then max_depth bounce launches
            // (each takes every ray of its input queue; continuing rays go to the other queue)
            rt::KWave w{};
            w.p = k;
            w.cap = wcap;
            for (uint32_t c0 = 0; c0 < k.n_items; c0 += wcap) {
                w.item_begin = c0;
                w.n_chunk = std::min(wcap, k.n_items - c0);
                w.out = wqa;
                RT_HIP(rt::launch_wave_gen(w, xst));
                rt::RayQueue qi = wqa, qo = wqb;
                for (uint32_t b = 0; b < std::max(1u, P.max_depth); ++b) {
                    RT_HIP(hipMemsetAsync(qo.count, 0, sizeof(uint32_t), xst));
                    w.in = qi;
                    w.out = qo;
                    RT_HIP(rt::launch_wave_bounce(cull_mode, w, static_cast<uint32_t>(wgrid), xst));
                    std::swap(qi, qo);
                }
            }
        } else {
            RT_HIP(rt::launch_render(variant, cull_mode, k, grid, xst));
            if (two_part) {
                if (!sc->ev_main[wb]) RT_HIP(hipEventCreateWithFlags(&sc->ev_main[wb], hipEventDisableTiming));
                RT_HIP(hipEventRecord(sc->ev_main[wb], xst));
            }
            if (k.deep_depth) {  // the deep launch: the queued paths, same grid, same stream
                rt::KParams kd = k;
                kd.deep_mode = k.deep_depth;
                kd.deep_depth = 0;
                // the deep paths bounce inside glass spheres, inside the box over all clusters:
                // the level-3 gate only costs there (alike within box noise, fewer box tests;
                // same bits)
                kd.use_root = deep_root_box_env() ? k.use_root : 0u;
                kd.deep_prio = deep_prio_env();
                // the shading records in LDS for the deep launch of a pass issued alone: its
                // paths bounce in glass and shade every segment, and its few busy waves wait on
                // each global round trip (config 3 single frame: deep launch 0.59 vs 0.65 ms).
                // Not beside other renders: its larger workgroups then displace theirs (frame
                // stream 2.69-2.73 vs 2.57-2.59 ms per frame, 8-way share 0.45 vs 0.42)
                if (deep_shade_lds_env() && !in_flight && variant != rt::V_EXACT_SCALAR && !k.shade_lds &&
                    static_cast<size_t>(k.blob_units) * 16u + kRenderStaticLds <= sc->max_lds) {
                    kd.shade_lds = 1u;
                    kd.lds_units = k.blob_units;
                }
                if (variant == rt::V_STATS_LDS && std::getenv("RT_DEBUG_DEEP_ONLY")) {
                    // diagnostics: the counters and events of the deep launch alone
                    RT_HIP(hipMemsetAsync(sc->dbg, 0, 16 * sizeof(unsigned long long), xst));
                    RT_HIP(hipMemsetAsync(sc->dbg + rt::kDbgEvBase, 0, rt::kDbgEvents * sizeof(unsigned long long), xst));
                }
                RT_HIP(rt::launch_render(variant, cull_mode, kd, grid, xst));
            }
        }
        if (variant == rt::V_STATS_LDS) sc->dbg_waves = grid * 4u;
        if (s1 == P.spp) RT_HIP(hipEventRecord(sc->ev_end[ring], xst));
        if (pipe) {
            RT_HIP(hipEventRecord(sc->ev_done[wb], xst));
            sc->last_ws = static_cast<int>(wb);
        }
        rt::KAccum a{};
        a.slots = sc->slots[wb];
        a.acc = sc->acc;
        a.out = d_rgb;
        a.out_u8 = nullptr;
        a.n_pixels = k.n_pixels;
        a.n_samples = s1 - s0;
        a.n_blocks = (std::min(s1, full_blocks_end) - std::min(s0, full_blocks_end)) / 4u;
        a.first = s0 == 0;
        a.last = s1 == P.spp;
        a.spp = P.spp;
        a.W = P.width;
        a.tiles_x = k.tiles_x;
        a.tiled_rows = k.tiled_rows;
        a.tile_lw = k.tile_lw;
        a.row_offset = k.row_offset;
        a.row_stride = k.row_stride;
        a.full_frame = k.full_frame;
        if (pipe && d_segments) a.seg_from = seg_b, a.seg_to = reinterpret_cast<unsigned long long *>(d_segments);
        a.queue_reset = k.queue_ctr;
        a.queue_words = 8 * rt::kQueueStride;
        if (k.deep_depth) {
            a.deep_over = sc->deep_over_dev + wb;
            a.deep_key = deep_key;
            a.deep_rcap = k.deep.rcap;
        }
        if (two_part) {
            // a pass issued while no other render runs (a lone frame, the first of a stream):
            // the pixels without deep samples accumulate beside the deep launch, the others (and
            // the counters) after it. In a frame stream the other frames' work fills that time,
            // and the extra launch per pass measured ~1% slower there.
            rt::KAccum a1 = a;
            a1.seg_from = a1.seg_to = nullptr;
            a1.queue_reset = nullptr;
            a1.deep_over = nullptr;
            a1.deep_px = k.deep.px;
            a1.part = 1;
            RT_HIP(hipStreamWaitEvent(st, sc->ev_main[wb], 0));
            RT_HIP(rt::launch_accumulate(a1, st));
            a.deep_px = k.deep.px;
            a.part = 2;
        } else if (k.deep_depth) {
            a.deep_px = k.deep.px;  // one part; clears the flags the main launch set
            a.part = 3;
        }
        if (pipe) RT_HIP(hipStreamWaitEvent(st, sc->ev_done[wb], 0));
        RT_HIP(rt::launch_accumulate(a, st));
        sc->ctr_dirty[wb] = false;
        if (pipe) {
            RT_HIP(hipEventRecord(sc->ev_free[wb], st));
            sc->free_valid[wb] = true;
        }
    }
    return RT_OK;
}

int render_compat(rt_scene *sc, const rt_camera *camera, const rt_params &P, float *d_rgb, hipStream_t st,
                  uint64_t *d_segments)
{
    rt::KCompat k{};
    for (int c = 0; c < 3; ++c) {
        k.org[c] = camera->origin[c];
        k.llc[c] = camera->lower_left_corner[c];
        k.hor[c] = camera->horizontal[c];
        k.ver[c] = camera->vertical[c];
    }
    k.W = P.width;
    k.H = P.height;
    k.spp = P.spp;
    k.max_depth = P.max_depth;
    k.row_offset = P.row_offset;
    k.row_stride = P.row_stride ? P.row_stride : 1;
    k.num_rows = rows_of(P);
    k.full_frame = (P.flags & RT_FLAG_FULL_FRAME) ? 1u : 0u;
    k.seed = static_cast<uint32_t>(P.seed);
    k.n_spheres = sc->n_spheres;
    const uint64_t n_pixels = static_cast<uint64_t>(P.width) * k.num_rows;
    if (n_pixels == 0) return RT_OK;
    if (n_pixels >= (1ull << 31)) return fail(RT_ERR_INVALID, "rt_render_device: more than 2^31 pixels in one call");
    k.n_pixels = static_cast<uint32_t>(n_pixels);
    k.n_chunks = (k.n_pixels + 63u) / 64u;
    k.shade = reinterpret_cast<const float4 *>(sc->blob[0]) + sc->shade_offset[0];
    k.out = d_rgb;
    k.ctr = sc->queue_ctr + kCompatCtr;
    k.segments = reinterpret_cast<unsigned long long *>(d_segments);
    int occ = 0;
    RT_HIP(rt::occupancy_compat(&occ));
    const uint32_t grid = static_cast<uint32_t>(
        std::max<uint64_t>(1, std::min<uint64_t>(static_cast<uint64_t>(std::max(occ, 1)) * sc->cu_count, (n_pixels + 255u) / 256u)));
    const uint32_t ring = static_cast<uint32_t>(sc->calls % rt_scene::kRing);
    ++sc->calls;
    RT_HIP(hipMemsetAsync(k.ctr, 0, sizeof(uint32_t), st));
    RT_HIP(hipEventRecord(sc->ev_begin[ring], st));
    RT_HIP(rt::launch_compat(k, grid, st));
    RT_HIP(hipEventRecord(sc->ev_end[ring], st));
    return RT_OK;
}
} // namespace

extern "C" {

int rt_render_cuda_impl(uint32_t width, uint32_t height, uint8_t *rgb_out)
{
    if (!rgb_out) return fail(RT_ERR_INVALID, "rt_render_cuda_impl: null output");
    rt_sphere s[8];
    rt_material m[8];
    uint32_t ns = 0, nm = 0;
    if (int rc = rt_scene_cuda(s, 8, &ns, m, 8, &nm); rc) return rc;
    rt_camera cam;
    if (int rc = rt_camera_cuda(width, height, &cam); rc) return rc;
    rt_params p{width, height, 48, 32, 0, 0, 1, 0, RT_FLAG_CUDA_COMPAT};  // cuda_impl.cu:62-63
    return rt_render_rgb8(s, ns, m, nm, &cam, &p, rgb_out, nullptr);
}

} // extern "C"

int rt_scene_kernel_times(rt_scene *sc, uint32_t max, float *ms, uint32_t *n)
{
    if (!sc || !n || (max && !ms)) return fail(RT_ERR_INVALID, "rt_scene_kernel_times: null argument");
    const uint64_t avail = std::min<uint64_t>(sc->calls, rt_scene::kRing);
    const uint32_t cnt = static_cast<uint32_t>(std::min<uint64_t>(avail, max));
    RT_HIP(hipSetDevice(sc->device));
    for (uint32_t i = 0; i < cnt; ++i) {
        const uint32_t r = static_cast<uint32_t>((sc->calls - cnt + i) % rt_scene::kRing);
        RT_HIP(hipEventSynchronize(sc->ev_end[r]));
        RT_HIP(hipEventElapsedTime(ms + i, sc->ev_begin[r], sc->ev_end[r]));
    }
    *n = cnt;
    return RT_OK;
}

int rt_scene_debug_counters(rt_scene *sc, uint64_t out[16], int reset)
{
    if (!sc || !out) return fail(RT_ERR_INVALID, "rt_scene_debug_counters: null argument");
    RT_HIP(hipSetDevice(sc->device));
    if (!sc->dbg) {
        std::memset(out, 0, 16 * sizeof(uint64_t));
        return RT_OK;
    }
    RT_HIP(hipDeviceSynchronize());
    RT_HIP(hipMemcpy(out, sc->dbg, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (reset) RT_HIP(hipMemset(sc->dbg, 0, 16 * sizeof(uint64_t)));
    return RT_OK;
}

int rt_scene_debug_events(rt_scene *sc, uint64_t out[32], int reset)
{
    if (!sc || !out) return fail(RT_ERR_INVALID, "rt_scene_debug_events: null argument");
    RT_HIP(hipSetDevice(sc->device));
    std::memset(out, 0, 32 * sizeof(uint64_t));
    if (!sc->dbg) return RT_OK;
    RT_HIP(hipDeviceSynchronize());
    RT_HIP(hipMemcpy(out, sc->dbg + rt::kDbgEvBase, rt::kDbgEvents * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (reset) RT_HIP(hipMemset(sc->dbg + rt::kDbgEvBase, 0, rt::kDbgEvents * sizeof(uint64_t)));
    return RT_OK;
}

int rt_scene_debug_timeline(rt_scene *sc, uint64_t *out, uint32_t max_waves, uint32_t *n)
{
    if (!sc || !out || !n) return fail(RT_ERR_INVALID, "rt_scene_debug_timeline: null argument");
    RT_HIP(hipSetDevice(sc->device));
    *n = 0;
    if (!sc->dbg) return RT_OK;
    const uint32_t waves = std::min({max_waves, sc->dbg_waves, rt::kDbgWaves});
    RT_HIP(hipDeviceSynchronize());
    RT_HIP(hipMemcpy(out, sc->dbg + 16, 4 * static_cast<size_t>(waves) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    *n = waves;
    return RT_OK;
}

int rt_epilogue_rgb8_device(const float *d_rgb, uint8_t *d_out, uint64_t n_pixels, void *stream)
{
    if (!d_rgb || !d_out) return fail(RT_ERR_INVALID, "rt_epilogue_rgb8_device: null argument");
    if (!n_pixels) return RT_OK;
    RT_HIP(rt::launch_epilogue(d_rgb, d_out, n_pixels * 3u, static_cast<hipStream_t>(stream)));
    return RT_OK;
}

} // extern "C"

namespace {

// Synchronous host-buffer render on the current device (the cuda_impl replacement).
int render_host(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                const rt_camera *camera, const rt_params *params, float *rgb_out, uint8_t *u8_out, rt_stats *stats)
{
    if (!camera || (!rgb_out && !u8_out)) return fail(RT_ERR_INVALID, "render: null argument");
    if (int rc = check_params(params); rc != RT_OK) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    int dev = 0;
    RT_HIP(hipGetDevice(&dev));
    rt_scene *sc = nullptr;
    if (int rc = rt_scene_create(spheres, n_spheres, materials, n_materials, dev, &sc); rc) return rc;
    const rt_params &P = *params;
    const uint64_t rows = (P.flags & RT_FLAG_FULL_FRAME) ? P.height : rows_of(P);
    const uint64_t n_values = rows * P.width * 3u;
    float *d_rgb = nullptr;
    uint8_t *d_u8 = nullptr;
    uint64_t *d_seg = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = RT_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == RT_OK) rc = fail(RT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
        return rc == RT_OK;
    };
    if (chk(hipMalloc((void **)&d_rgb, n_values * 4), "hipMalloc") && u8_out) chk(hipMalloc((void **)&d_u8, n_values), "hipMalloc");
    if (rc == RT_OK) chk(hipMalloc((void **)&d_seg, 24), "hipMalloc");
    if (rc == RT_OK && (P.flags & RT_FLAG_FULL_FRAME)) chk(hipMemset(d_rgb, 0, n_values * 4), "hipMemset");
    if (rc == RT_OK) chk(hipMemset(d_seg, 0, 24), "hipMemset");
    if (rc == RT_OK) chk(hipEventCreate(&e0), "hipEventCreate");
    if (rc == RT_OK) chk(hipEventCreate(&e1), "hipEventCreate");
    if (rc == RT_OK) chk(hipEventRecord(e0, nullptr), "hipEventRecord");
    if (rc == RT_OK) rc = rt_render_device(sc, camera, params, d_rgb, nullptr, d_seg);
    if (rc == RT_OK) chk(hipEventRecord(e1, nullptr), "hipEventRecord");
    if (rc == RT_OK && u8_out) rc = rt_epilogue_rgb8_device(d_rgb, d_u8, n_values / 3, nullptr);
    if (rc == RT_OK) chk(hipDeviceSynchronize(), "render");
    uint64_t segs[3] = {0, 0, 0};
    float ms = 0.f;
    if (rc == RT_OK && rgb_out) chk(hipMemcpy(rgb_out, d_rgb, n_values * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == RT_OK && u8_out) chk(hipMemcpy(u8_out, d_u8, n_values, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == RT_OK) chk(hipMemcpy(segs, d_seg, 24, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == RT_OK) chk(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (d_rgb) (void)hipFree(d_rgb);
    if (d_u8) (void)hipFree(d_u8);
    if (d_seg) (void)hipFree(d_seg);
    rt_scene_destroy(sc);
    if (rc == RT_OK && stats) {
        stats->primaries = static_cast<uint64_t>(P.width) * rows_of(P) * P.spp;
        stats->segments = segs[0];
        stats->sphere_tests = segs[1];
        stats->box_tests = segs[2];
        stats->kernel_ms = ms;
        stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return rc;
}

} // namespace

extern "C" {

int rt_render_f32(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                  const rt_camera *camera, const rt_params *params, float *rgb_out, rt_stats *stats)
{
    if (!rgb_out) return fail(RT_ERR_INVALID, "rt_render_f32: null output");
    return render_host(spheres, n_spheres, materials, n_materials, camera, params, rgb_out, nullptr, stats);
}

int rt_render_rgb8(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                   const rt_camera *camera, const rt_params *params, uint8_t *rgb_out, rt_stats *stats)
{
    if (!rgb_out) return fail(RT_ERR_INVALID, "rt_render_rgb8: null output");
    return render_host(spheres, n_spheres, materials, n_materials, camera, params, nullptr, rgb_out, stats);
}

} // extern "C"

// ---- single-process multi-GPU render: interleaved row tiles + RCCL gather over xGMI -----
// RCCL is opened with dlopen (librccl.so.1) on first use, so the library has no link-time
// dependency on it and shares the process's RCCL if another component (torch) loaded it.
namespace {
struct rccl_api {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok = false;
};
const rccl_api &rccl()
{
    static rccl_api api = [] {
        rccl_api a;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
        a.comm_init_all = reinterpret_cast<decltype(a.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
        a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        a.send = reinterpret_cast<decltype(a.send)>(dlsym(h, "ncclSend"));
        a.recv = reinterpret_cast<decltype(a.recv)>(dlsym(h, "ncclRecv"));
        a.group_start = reinterpret_cast<decltype(a.group_start)>(dlsym(h, "ncclGroupStart"));
        a.group_end = reinterpret_cast<decltype(a.group_end)>(dlsym(h, "ncclGroupEnd"));
        a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(h, "ncclGetErrorString"));
        a.ok = a.comm_init_all && a.comm_destroy && a.send && a.recv && a.group_start && a.group_end && a.error_string;
        return a;
    }();
    return api;
}
} // namespace

// Persistent multi-GPU context (rt_multi_*): rank r of N renders the rows y = r, r + N, ...
// (interleaved single rows balance sky against ground) on its device into a packed tile;
// optionally the gamma/u8 epilogue runs on the tile (3 B per pixel instead of 12 over xGMI);
// the tiles are gathered to rank 0's device and de-interleaved into the caller's frame.
// Everything that does not depend on the frame is built once at rt_multi_create: per-device
// scenes, rank streams, the RCCL communicators (ncclCommInitAll over the distinct devices), the
// segment counters; tiles and the gather buffer grow on first use of a frame size. Ranks that
// share a device with rank 0 ("virtual ranks": a one-GPU rehearsal of an N-way split) move
// their tile with a device copy where RCCL would send/recv; the tile layout, the gather buffer
// and the de-interleave are the same code either way.
struct rt_multi {
    int n = 0;
    std::vector<int> dev;
    bool rccl = false;  // every rank on its own device: gather over RCCL
    std::vector<rt_scene *> sc;
    std::vector<hipStream_t> st;        // rank r > 0: its stream (rank 0 runs on the caller's stream)
    std::vector<ncclComm_t> comm;
    std::vector<void *> tile;           // f32 tile per rank, on its device
    std::vector<size_t> tile_bytes;
    std::vector<void *> tile8;          // u8 tile per rank (RT_OUTPUT_RGB8)
    std::vector<size_t> tile8_bytes;
    std::vector<uint64_t *> seg;        // per rank: {segments, sphere tests, box tests}
    void *gather = nullptr;             // on rank 0's device: N slots of the largest tile
    size_t gather_bytes = 0;
    std::vector<hipEvent_t> ev_ready;   // virtual rank r: its tile is complete
    hipEvent_t ev_copied = nullptr;     // caller stream: virtual ranks' tiles copied out
    bool copied_valid = false;
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;
};

namespace {

int multi_fail_destroy(rt_multi *m, int rc);

// ensure() on a given device. Growing reallocates and so synchronises that device; the
// buffers of a context grow only when a frame is larger than any before it (rt_api.h)
int grow(int device, void **ptr, size_t *have, size_t want)
{
    if (*have >= want && *ptr) return RT_OK;
    RT_HIP(hipSetDevice(device));
    if (*ptr) {
        RT_HIP(hipDeviceSynchronize());
        RT_HIP(hipFree(*ptr));
        *ptr = nullptr;
        *have = 0;
    }
    RT_HIP(hipMalloc(ptr, std::max<size_t>(want, 256)));
    *have = want;
    return RT_OK;
}

uint32_t multi_rows(uint32_t H, int n, int r)
{
    return static_cast<uint32_t>(r) < H ? (H - static_cast<uint32_t>(r) + static_cast<uint32_t>(n) - 1) / static_cast<uint32_t>(n) : 0u;
}

} // namespace

extern "C" {

int rt_multi_create(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                    const int *devices, int n_ranks, rt_multi **out)
{
    if (!out) return fail(RT_ERR_INVALID, "rt_multi_create: null output");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_ERR_DEVICE, "rt_multi_create: no HIP device");
    const int N = n_ranks <= 0 ? ndev : n_ranks;
    if (!devices && N > ndev) return fail(RT_ERR_INVALID, "rt_multi_create: more ranks than devices (pass a device list)");
    if (N > 64) return fail(RT_ERR_INVALID, "rt_multi_create: at most 64 ranks");
    rt_multi *m = new rt_multi();
    m->n = N;
    for (int r = 0; r < N; ++r) {
        const int d = devices ? devices[r] : r;
        if (d < 0 || d >= ndev) {
            delete m;
            return fail(RT_ERR_INVALID, "rt_multi_create: bad device index");
        }
        m->dev.push_back(d);
    }
    // two supported layouts: every rank on its own device (RCCL), or every rank on rank 0's
    // device (virtual ranks); a mix would gather through cross-device copies no test covers
    bool distinct = true, all_same = true;
    for (int r = 1; r < N; ++r) {
        all_same = all_same && m->dev[r] == m->dev[0];
        for (int q = 0; q < r; ++q) distinct = distinct && m->dev[q] != m->dev[r];
    }
    if (!distinct && !all_same) {
        delete m;
        return fail(RT_ERR_INVALID, "rt_multi_create: devices must be all distinct or all rank 0's device");
    }
    m->rccl = N > 1 && distinct;
    m->sc.assign(N, nullptr);
    m->st.assign(N, nullptr);
    m->tile.assign(N, nullptr);
    m->tile_bytes.assign(N, 0);
    m->tile8.assign(N, nullptr);
    m->tile8_bytes.assign(N, 0);
    m->seg.assign(N, nullptr);
    m->ev_ready.assign(N, nullptr);
    int rc = RT_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == RT_OK) rc = fail(RT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
        return rc == RT_OK;
    };
    for (int r = 0; r < N && rc == RT_OK; ++r) {
        rc = rt_scene_create(spheres, n_spheres, materials, n_materials, m->dev[r], &m->sc[r]);
        if (rc != RT_OK) break;
        chk(hipSetDevice(m->dev[r]), "hipSetDevice");
        if (r > 0) chk(hipStreamCreateWithFlags(&m->st[r], hipStreamNonBlocking), "hipStreamCreate");
        chk(hipMalloc((void **)&m->seg[r], 3 * sizeof(uint64_t)), "hipMalloc");
        chk(hipMemset(m->seg[r], 0, 3 * sizeof(uint64_t)), "hipMemset");
        chk(hipEventCreateWithFlags(&m->ev_ready[r], hipEventDisableTiming), "hipEventCreate");
    }
    if (rc == RT_OK) {
        chk(hipSetDevice(m->dev[0]), "hipSetDevice");
        chk(hipEventCreateWithFlags(&m->ev_copied, hipEventDisableTiming), "hipEventCreate");
        chk(hipEventCreate(&m->ev_t0), "hipEventCreate");
        chk(hipEventCreate(&m->ev_t1), "hipEventCreate");
    }
    if (rc == RT_OK && m->rccl) {
        const rccl_api &api = rccl();
        if (!api.ok) {
            rc = fail(RT_ERR_COMM, "rt_multi_create: librccl.so.1 not loadable");
        } else {
            m->comm.assign(N, nullptr);
            const ncclResult_t nr = api.comm_init_all(m->comm.data(), N, m->dev.data());
            if (nr != ncclSuccess) {
                m->comm.clear();
                rc = fail(RT_ERR_COMM, std::string("ncclCommInitAll: ") + api.error_string(nr));
            }
        }
    }
    if (rc != RT_OK) return multi_fail_destroy(m, rc);
    (void)hipSetDevice(m->dev[0]);
    *out = m;
    return RT_OK;
}

int rt_multi_destroy(rt_multi *m)
{
    if (!m) return RT_OK;
    for (int r = 0; r < m->n; ++r) {
        (void)hipSetDevice(m->dev[r]);
        if (m->st[r]) (void)hipStreamSynchronize(m->st[r]);
    }
    (void)hipSetDevice(m->dev[0]);
    (void)hipDeviceSynchronize();
    for (auto c : m->comm)
        if (c) rccl().comm_destroy(c);
    for (int r = 0; r < m->n; ++r) {
        (void)hipSetDevice(m->dev[r]);
        if (m->tile[r]) (void)hipFree(m->tile[r]);
        if (m->tile8[r]) (void)hipFree(m->tile8[r]);
        if (m->seg[r]) (void)hipFree(m->seg[r]);
        if (m->ev_ready[r]) (void)hipEventDestroy(m->ev_ready[r]);
        if (m->st[r]) (void)hipStreamDestroy(m->st[r]);
        if (m->sc[r]) rt_scene_destroy(m->sc[r]);
    }
    (void)hipSetDevice(m->dev[0]);
    if (m->gather) (void)hipFree(m->gather);
    for (hipEvent_t e : {m->ev_copied, m->ev_t0, m->ev_t1})
        if (e) (void)hipEventDestroy(e);
    delete m;
    return RT_OK;
}

int rt_multi_info(const rt_multi *m, int *n_ranks, int *uses_rccl)
{
    if (!m) return fail(RT_ERR_INVALID, "rt_multi_info: null context");
    if (n_ranks) *n_ranks = m->n;
    if (uses_rccl) *uses_rccl = m->rccl ? 1 : 0;
    return RT_OK;
}

int rt_multi_render_device(rt_multi *m, const rt_camera *camera, const rt_params *params, uint32_t format,
                           void *d_out, void *stream)
{
    if (!m || !camera || !d_out) return fail(RT_ERR_INVALID, "rt_multi_render_device: null argument");
    if (format != RT_OUTPUT_F32 && format != RT_OUTPUT_RGB8) return fail(RT_ERR_INVALID, "rt_multi_render_device: bad format");
    if (int rc = check_params(params); rc != RT_OK) return rc;
    const rt_params base = *params;
    const int N = m->n;
    const uint32_t W = base.width, H = base.height;
    const size_t es = format == RT_OUTPUT_F32 ? 4u : 1u;
    const size_t row_vals = static_cast<size_t>(W) * 3u;
    const uint32_t rows_max = multi_rows(H, N, 0);
    hipStream_t cs = static_cast<hipStream_t>(stream);
    // buffers (grow only: a new, larger frame size costs one synchronisation)
    for (int r = 0; r < N; ++r) {
        const size_t rows = multi_rows(H, N, r);
        if (int rc = grow(m->dev[r], &m->tile[r], &m->tile_bytes[r], std::max<size_t>(rows, 1) * row_vals * 4u); rc) return rc;
        if (format == RT_OUTPUT_RGB8)
            if (int rc = grow(m->dev[r], &m->tile8[r], &m->tile8_bytes[r], std::max<size_t>(rows, 1) * row_vals); rc) return rc;
    }
    if (N > 1)
        if (int rc = grow(m->dev[0], &m->gather, &m->gather_bytes, static_cast<size_t>(N) * rows_max * row_vals * es); rc)
            return rc;
    auto tile_of = [&](int r) -> void * { return format == RT_OUTPUT_F32 ? m->tile[r] : m->tile8[r]; };
    // 1. every rank renders its rows (rank 0 on the caller's stream); virtual ranks wait until
    //    the caller stream has copied their previous tile out
    for (int r = 0; r < N; ++r) {
        const uint32_t rows = multi_rows(H, N, r);
        if (!rows) continue;
        rt_params p = base;
        p.row_offset = static_cast<uint32_t>(r);
        p.row_stride = static_cast<uint32_t>(N);
        p.num_rows = rows;
        p.flags &= ~static_cast<uint32_t>(RT_FLAG_FULL_FRAME);
        hipStream_t rs = r == 0 ? cs : m->st[r];
        RT_HIP(hipSetDevice(m->dev[r]));
        if (r > 0 && !m->rccl && m->copied_valid) RT_HIP(hipStreamWaitEvent(rs, m->ev_copied, 0));
        if (int rc = rt_render_device(m->sc[r], camera, &p, static_cast<float *>(m->tile[r]), rs, m->seg[r]); rc) return rc;
        if (format == RT_OUTPUT_RGB8)
            RT_HIP(rt::launch_epilogue(static_cast<const float *>(m->tile[r]), static_cast<uint8_t *>(m->tile8[r]),
                                       static_cast<uint64_t>(rows) * row_vals, rs));
        if (r > 0 && !m->rccl) RT_HIP(hipEventRecord(m->ev_ready[r], rs));
    }
    // 2. the gather: tile r -> slot r of the gather buffer on rank 0's device
    const size_t slot_bytes = static_cast<size_t>(rows_max) * row_vals * es;
    if (N > 1 && m->rccl) {
        const rccl_api &api = rccl();
        ncclResult_t nr = api.group_start();
        for (int r = 1; r < N && nr == ncclSuccess; ++r) {
            const size_t cnt = static_cast<size_t>(multi_rows(H, N, r)) * row_vals;
            if (!cnt) continue;
            const ncclDataType_t ty = format == RT_OUTPUT_F32 ? ncclFloat : ncclUint8;
            nr = api.send(tile_of(r), cnt, ty, 0, m->comm[r], m->st[r]);
            if (nr == ncclSuccess)
                nr = api.recv(static_cast<char *>(m->gather) + r * slot_bytes, cnt, ty, r, m->comm[0], cs);
        }
        const ncclResult_t ne = api.group_end();
        if (nr == ncclSuccess) nr = ne;
        if (nr != ncclSuccess) return fail(RT_ERR_COMM, std::string("RCCL gather: ") + api.error_string(nr));
    } else if (N > 1) {
        RT_HIP(hipSetDevice(m->dev[0]));
        for (int r = 1; r < N; ++r) {
            const size_t bytes = static_cast<size_t>(multi_rows(H, N, r)) * row_vals * es;
            if (!bytes) continue;
            RT_HIP(hipStreamWaitEvent(cs, m->ev_ready[r], 0));
            RT_HIP(hipMemcpyAsync(static_cast<char *>(m->gather) + r * slot_bytes, tile_of(r), bytes,
                                  hipMemcpyDeviceToDevice, cs));
        }
        RT_HIP(hipEventRecord(m->ev_copied, cs));
        m->copied_valid = true;
    }
    // 3. de-interleave on rank 0's device: frame row r + i N <- tile r row i
    RT_HIP(hipSetDevice(m->dev[0]));
    const size_t row_bytes = row_vals * es;
    for (int r = 0; r < N; ++r) {
        const uint32_t rows = multi_rows(H, N, r);
        if (!rows) continue;
        const void *src = r == 0 ? tile_of(0) : static_cast<const void *>(static_cast<char *>(m->gather) + r * slot_bytes);
        RT_HIP(hipMemcpy2DAsync(static_cast<char *>(d_out) + r * row_bytes, row_bytes * N, src, row_bytes, row_bytes,
                                rows, hipMemcpyDeviceToDevice, cs));
    }
    return RT_OK;
}

} // extern "C"

namespace {

int multi_fail_destroy(rt_multi *m, int rc)
{
    const std::string msg = g_error;
    rt_multi_destroy(m);
    g_error = msg;
    return rc;
}

// Synchronous host-buffer frame through a context: every rank's counters are zeroed, the frame
// is enqueued on an internal stream of rank 0's device, copied to `out` and timed.
int multi_render_host(rt_multi *m, const rt_camera *camera, const rt_params *params, uint32_t format, void *out,
                      rt_stats *stats)
{
    if (!m || !camera || !out) return fail(RT_ERR_INVALID, "rt_multi_render: null argument");
    if (int rc = check_params(params); rc != RT_OK) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    const size_t es = format == RT_OUTPUT_F32 ? 4u : 1u;
    const size_t bytes = static_cast<size_t>(params->width) * params->height * 3u * es;
    for (int r = 0; r < m->n; ++r) {
        RT_HIP(hipSetDevice(m->dev[r]));
        RT_HIP(hipMemset(m->seg[r], 0, 3 * sizeof(uint64_t)));
    }
    RT_HIP(hipSetDevice(m->dev[0]));
    void *d_out = nullptr;
    hipStream_t cs = nullptr;
    RT_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    int rc = RT_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == RT_OK) rc = fail(RT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
        return rc == RT_OK;
    };
    chk(hipMalloc(&d_out, bytes), "hipMalloc");
    if (rc == RT_OK) chk(hipEventRecord(m->ev_t0, cs), "hipEventRecord");
    if (rc == RT_OK) rc = rt_multi_render_device(m, camera, params, format, d_out, cs);
    (void)hipSetDevice(m->dev[0]);
    if (rc == RT_OK) chk(hipEventRecord(m->ev_t1, cs), "hipEventRecord");
    if (rc == RT_OK) chk(hipMemcpyAsync(out, d_out, bytes, hipMemcpyDeviceToHost, cs), "hipMemcpyAsync");
    for (int r = 0; r < m->n; ++r) {
        (void)hipSetDevice(m->dev[r]);
        if (m->st[r]) chk(hipStreamSynchronize(m->st[r]), "hipStreamSynchronize");
    }
    (void)hipSetDevice(m->dev[0]);
    chk(hipStreamSynchronize(cs), "hipStreamSynchronize");
    uint64_t segs[3] = {0, 0, 0};
    for (int r = 0; r < m->n && rc == RT_OK; ++r) {
        uint64_t v[3];
        (void)hipSetDevice(m->dev[r]);
        chk(hipMemcpy(v, m->seg[r], sizeof v, hipMemcpyDeviceToHost), "hipMemcpy");
        for (int i = 0; i < 3; ++i) segs[i] += v[i];
    }
    (void)hipSetDevice(m->dev[0]);
    float ms = 0.f;
    if (rc == RT_OK) chk(hipEventElapsedTime(&ms, m->ev_t0, m->ev_t1), "hipEventElapsedTime");
    if (d_out) (void)hipFree(d_out);
    (void)hipStreamDestroy(cs);
    if (rc == RT_OK && stats) {
        stats->primaries = static_cast<uint64_t>(params->width) * params->height * params->spp;
        stats->segments = segs[0];
        stats->sphere_tests = segs[1];
        stats->box_tests = segs[2];
        stats->kernel_ms = ms;
        stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return rc;
}

int render_multi_once(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                      const rt_camera *camera, const rt_params *params, int ngpu, uint32_t format, void *out,
                      rt_stats *stats)
{
    if (!camera || !out) return fail(RT_ERR_INVALID, "rt_render_multi: null argument");
    if (int rc = check_params(params); rc != RT_OK) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_ERR_DEVICE, "rt_render_multi: no HIP device");
    rt_multi *m = nullptr;
    if (int rc = rt_multi_create(spheres, n_spheres, materials, n_materials, nullptr,
                                 ngpu <= 0 ? ndev : std::min(ngpu, ndev), &m); rc)
        return rc;
    const int rc = multi_render_host(m, camera, params, format, out, stats);
    const std::string msg = g_error;
    rt_multi_destroy(m);
    g_error = msg;
    return rc;
}

} // namespace

extern "C" {

int rt_multi_render_f32(rt_multi *m, const rt_camera *camera, const rt_params *params, float *rgb_out, rt_stats *stats)
{
    return multi_render_host(m, camera, params, RT_OUTPUT_F32, rgb_out, stats);
}

int rt_multi_render_rgb8(rt_multi *m, const rt_camera *camera, const rt_params *params, uint8_t *rgb_out,
                         rt_stats *stats)
{
    return multi_render_host(m, camera, params, RT_OUTPUT_RGB8, rgb_out, stats);
}

int rt_render_multi_f32(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials,
                        uint32_t n_materials, const rt_camera *camera, const rt_params *params, int ngpu,
                        float *rgb_out, rt_stats *stats)
{
    return render_multi_once(spheres, n_spheres, materials, n_materials, camera, params, ngpu, RT_OUTPUT_F32, rgb_out,
                             stats);
}

int rt_render_multi_rgb8(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials,
                         uint32_t n_materials, const rt_camera *camera, const rt_params *params, int ngpu,
                         uint8_t *rgb_out, rt_stats *stats)
{
    return render_multi_once(spheres, n_spheres, materials, n_materials, camera, params, ngpu, RT_OUTPUT_RGB8, rgb_out,
                             stats);
}

// app::save_to_file, src/main.cxx:87-101: "P6\n<width> <height>\n255\n", then the texels.
int rt_write_ppm(const char *path, const uint8_t *rgb, uint32_t width, uint32_t height)
{
    if (!path || (!rgb && width && height)) return fail(RT_ERR_INVALID, "rt_write_ppm: null argument");
    std::FILE *f = std::fopen(path, "wb");
    if (!f) return fail(RT_ERR_IO, std::string("rt_write_ppm: bad file ") + path);
    const std::string hdr = "P6\n" + std::to_string(width) + " " + std::to_string(height) + "\n255\n";
    const size_t n = static_cast<size_t>(width) * height * 3u;
    const bool ok = std::fwrite(hdr.data(), 1, hdr.size(), f) == hdr.size() && (n == 0 || std::fwrite(rgb, 1, n, f) == n);
    const bool closed = std::fclose(f) == 0;
    if (!ok || !closed) return fail(RT_ERR_IO, std::string("rt_write_ppm: write failed: ") + path);
    return RT_OK;
}

} // extern "C"
