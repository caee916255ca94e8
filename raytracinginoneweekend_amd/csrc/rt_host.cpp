// rt_host.cpp — the device half of the C-ABI's host side (include/rt_api.h): device scene upload,
// pass planning under the scene's options, frames in flight, the render entry points that replace
// `cuda_impl` (src/main.cxx:18, src/CUDA/cuda_impl.cu:384) and the multi-GPU context. The
// host-only half (camera and scene constructors, cluster builder, options, PPM writer) is
// rt_host_build.cpp.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
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
#include "rt_host_build.h"

using namespace rthost;

namespace rt {
hipError_t launch_render(int variant, int cull, const KParams &p, uint32_t grid, hipStream_t stream, int wpb = 4);
#ifndef RT_LONE_DEEP_TMAX
#define RT_LONE_DEEP_TMAX 4u  // the lone deep launch's transposition threshold (below)
#endif
hipError_t deep_occupancy(int variant, int wpb, size_t lds, int *blocks_per_cu, size_t *static_lds);
hipError_t occupancy_render(int variant, int cull, int *blocks_per_cu, size_t lds, bool pairs = false);
hipError_t static_lds_render(int variant, int cull, size_t *bytes, bool pairs = false);
hipError_t launch_accumulate(const KAccum &k, hipStream_t stream);
hipError_t launch_compat(const KCompat &k, uint32_t grid, hipStream_t stream);
hipError_t launch_wave_gen(const KWave &w, hipStream_t stream);
hipError_t launch_wave_bounce(int cull, const KWave &w, uint32_t grid, hipStream_t stream);
hipError_t occupancy_wave_bounce(int cull, int *blocks_per_cu, size_t lds);
hipError_t occupancy_compat(int *blocks_per_cu);
hipError_t launch_epilogue(const float *in, uint8_t *out, uint64_t n, hipStream_t stream);
hipError_t launch_sky(const KSky &k, hipStream_t stream);
} // namespace rt

namespace {


#define RT_HIP(call)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(RT_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)


// counters: [kMaxWs][8 queues x kQueueStride], then [kMaxWs][4] u64 segment counters, then
// the compat kernel's counter
constexpr size_t kSegWords = kMaxWs * 8 * rt::kQueueStride;
constexpr size_t kCompatCtr = kSegWords + kMaxWs * 8 + 16;
constexpr size_t kCtrWords = kCompatCtr + rt::kQueueStride;


// Item dealing (guided): each queue's chunks shrink geometrically from 1/K of its remaining
// share per wave down to 128 items — few queue atomics, big coherent chunks for most of the
// launch, small ones at its end. Config 3 frame stream: K = 6 3.93 ms/frame with single-frame
// latency unchanged (5.3-5.4 ms); K = 4 3.89-3.92 but 6.2 ms latency; fixed 512-item chunks
// with a 64-item tail 4.39 ms (round 1; the fixed scheme was removed in round 4). A pass
// issued while no other render runs (a lone frame) deals with K = 12 — its end is not hidden
// by other launches, and smaller last chunks even it out (config 3 lone frame 3.37-3.45 vs
// 3.55-3.59 ms, frame stream alike at K = 6/9/12/16; profiles/r03/ab/guided_k.txt).
float guided_l2b(uint32_t total_waves, bool in_flight)
{
    const double k = in_flight ? 6.0 : 12.0;
    const double wq = std::max(1.0, total_waves / 8.0);
    const double beta = std::max(1.0 - 1.0 / (k * wq), 1.0 / (1 << 20));
    return static_cast<float>(std::log2(beta));
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
// the third applies to short passes only. Round 3 re-swept 3/5/7 (7 streams): the default best
// or within noise (profiles/r03/ab/knobs_s3.txt).
constexpr uint64_t kShortPassItems = 32ull << 20;
// the deep launch of a lone pass stages the shading records in LDS (A/B build switch)
// lone split passes accumulate in two parts, the first beside the deep launch (A/B build switch)
#ifndef RT_LONE_SKY_ROOM
#define RT_LONE_SKY_ROOM -1  // -1: by the sky's share of the pass (see the main launch's grid)
#endif
#ifndef RT_TWO_PART
#define RT_TWO_PART 1
#endif
#ifndef RT_DEEP_LDS_STAGE
#define RT_DEEP_LDS_STAGE 1
#endif
// ... in 8-wave workgroups (one LDS copy of the scene for twice the waves), every workgroup
// resident at once, dealing the queued paths statically (A/B build switches)
#ifndef RT_DEEP_WIDE
#define RT_DEEP_WIDE 1
#endif
#ifndef RT_DEEP_STATIC
#define RT_DEEP_STATIC 1
#endif
#ifndef RT_SHORT_OTHERS  // A/B build switch: the divisor for short passes in flight (-1: streams - 1)
#define RT_SHORT_OTHERS -1
#endif
int grid_wg_per_cu(int occ, bool in_flight, uint32_t streams, uint64_t pass_items)
{
    if (!in_flight) return occ;
    const int short_others = RT_SHORT_OTHERS > 0 ? RT_SHORT_OTHERS : std::max(1, static_cast<int>(streams) - 1);
    const int others = pass_items <= kShortPassItems ? short_others
                                                     : std::min(2, std::max(1, static_cast<int>(streams) - 1));
    return std::max(1, (occ + others - 1) / others);
}

} // namespace

struct rt_scene {
    int device = 0;
    rt_options opt{};  // fixed at creation (rt_scene_create_ex)
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
    // where the pair-arrival words of the queue of workspace w lay in its last layout (the
    // arrays' offsets follow the pixel count and the region capacity): zeroed again when moved
    size_t deep_meet_at[kMaxWs] = {};
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
    // the sky kernel of a pass issued alone runs beside the pass's main and deep launches, on the
    // next render stream (idle: nothing else runs); ev_sky after it
    hipEvent_t ev_sky = nullptr;
    bool free_valid[kMaxWs] = {};
    // queue/segment counters of workspace b not known to be zero (set while a render using
    // them is enqueued, cleared once the accumulation that resets them is enqueued after it)
    bool ctr_dirty[kMaxWs];
    rt_scene() { std::fill(std::begin(ctr_dirty), std::end(ctr_dirty), true); }
    uint32_t next_buf = 0;  // workspace of the next render pass
    int last_ws = -1;       // workspace of the last render pass issued (its ev_done), -1 = none
    // the caller stream of the previous call and an event after the last work enqueued on it:
    // a call on another stream first waits for it, so the shared accumulation buffer, the
    // compat counter and (render_streams = 1) the workspaces are never used by two streams at once
    hipStream_t last_stream = nullptr;
    hipEvent_t ev_tail = nullptr;
    bool tail_valid = false;
    int cu_count = 0;
    int occ[4][2][2];  // [variant][culled][shade records in LDS] blocks per CU, -1 = unknown
    int occ_pairs[4][2];  // the culled kernel's sample-pair instantiation, [variant][shade records in LDS]
    // [variant] blocks per CU of the 8-wave deep kernel with the whole blob in LDS, -1 = unknown,
    // 0 = it does not fit or holds no more waves than 4-wave groups (the lone deep launch)
    int occ_deep_wide[4] = {-1, -1, -1, -1};
    unsigned long long *dbg = nullptr;  // diagnostic counters (RT_DIAG_STATS)
    uint32_t dbg_waves = 0;             // waves of the last instrumented launch
    size_t max_lds = 0;
    // static LDS of the render kernel per traversal, [0] brute force, [1] culled (per-wave
    // transposed-test records and per-lane arrays; hipFuncGetAttributes)
    size_t static_lds[2] = {0, 0};
    size_t static_lds_pairs = 0;  // the culled kernel's sample-pair instantiation (its parked colours)
    // the last render's cut (rt_scene_usage_get)
    uint32_t used_streams = 0, used_ws = 0, used_pass = 0, used_deep = 0, used_pairs = 0, used_split = 0;
    uint32_t used_lead = 0, used_sky = 0;  // the last pass's tile classes
    // the culled scene's geometry for the tile classes of a pass, and the
    // dealing orders computed from it, per camera and rows (a pure function of those and the
    // scene, kept for the kOrders most recently used), each with its block permutation on the device
    rthost::scene_geom geom;
    bool has_geom = false;
    struct Order {
        std::vector<unsigned char> key;
        rthost::tile_order t;
        uint32_t *d_perm = nullptr;
        uint64_t used = 0;
    };
    static constexpr size_t kOrders = 8;
    std::vector<Order> orders;
    // ring of (start, end) events bracketing the render kernels of each rt_render_device call
    static constexpr uint32_t kRing = 256;
    std::vector<hipEvent_t> ev_begin, ev_end;
    uint64_t calls = 0;
};

extern "C" {


int rt_device_count(int *count)
{
    if (!count) return fail(RT_ERR_INVALID, "rt_device_count: null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return RT_OK;
}



} // extern "C"

namespace {



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
    f.n_pairs = k.n_pair_items / k.n_pixels;
}

bool camera_in_fast_range(const rt_camera &c)
{
    for (int i = 0; i < 3; ++i)
        for (float v : {c.origin[i], c.lower_left_corner[i], c.horizontal[i], c.vertical[i]})
            if (!(std::fabs(v) <= 0x1p19f)) return false;
    return std::fabs(c.lens_radius) <= 0x1p19f;
}

// deep queue of a pass: 8 regions of 1/1024 of its samples each (at least 512): 0.8% of the
// samples, where 0.2-0.3% reach the split depth on config 3; paths past a full region stay in the
// main launch. A pass of fewer than rt_options.deep_min_items samples (2^25) issued while no
// other render runs (a lone frame) is not split: its deep launch would be a serial tail of
// about max_depth - split iterations, which such a pass's own drain does not outweigh (config
// 3's 8-way row share alone: 1.28-1.30 ms split vs 1.03-1.10). Passes issued while others run
// (a frame stream) are split at any size: the unsplit drain costs issue (the 8-way share ran
// 42% more VALU instructions per sample than the full frame) and the deep launches run beside
// the other frames (8-way share, 7 streams: 0.50-0.51 ms per frame vs 0.58-0.59 unsplit).
uint32_t deep_region_cap(uint64_t n_samples)
{
    return static_cast<uint32_t>(std::max<uint64_t>(512u, n_samples / 1024u));
}
size_t deep_px_bytes(uint64_t n_pixels) { return (n_pixels + 255u) & ~static_cast<size_t>(255u); }
size_t deep_queue_bytes(uint64_t n_pixels, uint64_t n_samples)
{
    return deep_px_bytes(n_pixels) + static_cast<size_t>(8u) * deep_region_cap(n_samples) * 60u;
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

} // namespace

struct rt_scene;
namespace {

// RT_FLAG_CUDA_COMPAT: the reference's CUDA variant semantics (compat_kernel), on the caller
// stream, spheres read from the index-ordered shading records of the brute-force blob.
int render_compat(rt_scene *sc, const rt_camera *camera, const rt_params &P, float *d_rgb, hipStream_t st,
                  uint64_t *d_segments);

// Render streams (rt_options.render_streams): 1 runs the render kernels on the caller stream;
// 2..kMaxBufs rotate that many internal streams. 0 (auto): one stream fewer than the process's
// hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4; the caller's stream takes one), 2..7.
// The max-depth paths give every launch a drain of ~64 iterations whatever its size; with 3
// streams (and partial grids, grid_wg_per_cu) two other renders fill the machine while one
// drains. Measured on config 3 (frame stream): 3.81-3.87 ms/frame with 3 streams vs 3.90-3.93
// with 2; an 8-way row share (14.7 M samples) 0.63-0.64 vs 0.68. Round 3, with row shares split
// in flight: 7 streams beat 4 (config 3's 8-way share 0.50 vs 0.58 ms, 4-way 0.88 vs 0.95; the
// full frame 2.99-3.04 vs 3.06-3.08) and 8 (on 12 hardware queues) is slower again
// (profiles/r03/ab). More streams than hardware queues share queues and serialise.
uint32_t render_streams_of(const rt_options &o)
{
    if (o.render_streams) return o.render_streams;
    static const uint32_t hw_streams = [] {
        const char *q = std::getenv("GPU_MAX_HW_QUEUES");
        const unsigned long hw = q && *q ? std::strtoul(q, nullptr, 10) : 4ul;
        return static_cast<uint32_t>(std::clamp<unsigned long>(hw > 1 ? hw - 1 : 1, 2, 7));
    }();
    return hw_streams;
}


// *fresh (optional): set when the buffer was (re)allocated, whatever address it got back (the
// allocator may return the freed one; ADVICE r5: callers key their resets on this, not on the address)
int ensure(void **ptr, size_t *have, size_t want, bool *fresh = nullptr)
{
    if (fresh) *fresh = false;
    if (*have >= want && *ptr) return RT_OK;
    if (fresh) *fresh = true;
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

// frees every workspace of a scene (slots, deep queues, multi-pass sums, wavefront queues)
// after the device is idle: the next render re-cuts them under max_workspace_bytes
int free_workspaces(rt_scene *sc);

} // namespace

extern "C" {


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
    if (sc->ev_sky) (void)hipEventDestroy(sc->ev_sky);
    for (void *p : {(void *)sc->blob[0], (void *)sc->blob[1], (void *)sc->dbg, (void *)sc->acc, (void *)sc->queue_ctr, sc->wq})
        if (p) (void)hipFree(p);
    for (float *p : sc->slots)
        if (p) (void)hipFree(p);
    for (void *p : sc->deep)
        if (p) (void)hipFree(p);
    if (sc->deep_over) (void)hipHostFree(sc->deep_over);
    for (auto &o : sc->orders)
        if (o.d_perm) (void)hipFree(o.d_perm);
    (void)hipSetDevice(prev);
    delete sc;
    return RT_OK;
}

int rt_scene_create(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials,
                    uint32_t n_materials, int device, rt_scene **out)
{
    return rt_scene_create_ex(spheres, n_spheres, materials, n_materials, device, nullptr, out);
}

int rt_scene_create_ex(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials,
                       uint32_t n_materials, int device, const rt_options *options, rt_scene **out)
{
    if (!out || (n_spheres && !spheres) || !materials || !n_materials)
        return fail(RT_ERR_INVALID, "rt_scene_create: null argument or no materials");
    *out = nullptr;
    rt_options opt;
    if (options) {
        if (int rc = check_options(*options); rc) return rc;
        opt = *options;
    } else if (int rc = default_options(opt); rc) {
        return rc;
    }
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
    blob_t blobs[2] = {build_blob(spheres, n_spheres, false, opt.cluster_size),
                       build_blob(spheres, n_spheres, true, opt.cluster_size)};
    const std::vector<uint32_t> shortcut =
        shortcut_words(spheres, n_spheres, materials, blobs[1], (opt.diag & RT_DIAG_NO_NEIGHBOURS) != 0);
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
    sc->opt = opt;
    if (blobs[1].n_clusters) {
        sc->geom = scene_geometry(spheres, blobs[1]);
        sc->has_geom = true;
    }
    for (auto &r : sc->occ) for (auto &x : r) x[0] = x[1] = -1;
    for (auto &r : sc->occ_pairs) r[0] = r[1] = -1;
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
        if (rc == RT_OK && (hipEventCreateWithFlags(&sc->ev_tail, hipEventDisableTiming) != hipSuccess ||
                            hipEventCreateWithFlags(&sc->ev_sky, hipEventDisableTiming) != hipSuccess))
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
    if (rc == RT_OK) {
        hipError_t e = rt::static_lds_render(rt::V_EXACT_LDS, 0, &sc->static_lds[0]);
        if (e == hipSuccess) e = rt::static_lds_render(rt::V_EXACT_LDS, 7, &sc->static_lds[1]);
        if (e == hipSuccess) e = rt::static_lds_render(rt::V_EXACT_LDS, 7, &sc->static_lds_pairs, true);
        if (e != hipSuccess) rc = fail(RT_ERR_DEVICE, std::string("hipFuncGetAttributes: ") + hipGetErrorString(e));
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
// The dealing order of a pass over these rows with this camera (rt_scene::orders; computed on a
// miss: classify_tiles on the host, the permutation uploaded once).
int pass_order(rt_scene *sc, const rt_camera &cam, const rt::KParams &k, const rt_scene::Order **out)
{
    *out = nullptr;
    std::vector<unsigned char> key(sizeof(rt_camera) + 7 * sizeof(uint32_t));
    const uint32_t g[7] = {k.W, k.H, k.row_offset, k.row_stride, k.num_rows, k.tile_lw, 0u};
    std::memcpy(key.data(), &cam, sizeof(rt_camera));
    std::memcpy(key.data() + sizeof(rt_camera), g, sizeof(g));
    static uint64_t tick = 0;
    for (auto &o : sc->orders)
        if (o.key == key) {
            o.used = ++tick;
            *out = &o;
            return RT_OK;
        }
    rt_scene::Order e;
    e.key.swap(key);
    e.t = classify_tiles(cam, k.W, k.H, k.row_offset, k.row_stride, k.num_rows, k.tile_lw, sc->geom);
#ifdef RT_ORDER_IDENTITY  // A/B build switch: the class machinery over the natural order (one middle group)
    for (uint32_t i = 0; i < e.t.perm.size(); ++i) e.t.perm[i] = i;
    e.t.n_lead = e.t.n_sky = 0;
#endif
    if (!e.t.perm.empty()) {
        RT_HIP(hipMalloc((void **)&e.d_perm, e.t.perm.size() * sizeof(uint32_t)));
        const hipError_t ce = hipMemcpy(e.d_perm, e.t.perm.data(), e.t.perm.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
        if (ce != hipSuccess) {
            (void)hipFree(e.d_perm);
            return fail(RT_ERR_DEVICE, std::string("hipMemcpy: ") + hipGetErrorString(ce));
        }
    }
    if (sc->orders.size() >= rt_scene::kOrders) {
        auto lru = std::min_element(sc->orders.begin(), sc->orders.end(),
                                    [](const rt_scene::Order &a, const rt_scene::Order &b) { return a.used < b.used; });
        RT_HIP(hipDeviceSynchronize());  // renders in flight may still read its permutation
        if (lru->d_perm) RT_HIP(hipFree(lru->d_perm));
        sc->orders.erase(lru);
    }
    e.used = ++tick;
    sc->orders.push_back(std::move(e));
    *out = &sc->orders.back();
    return RT_OK;
}

int free_workspaces(rt_scene *sc)
{
    RT_HIP(hipDeviceSynchronize());
    auto drop = [](void *&p, size_t &n) -> hipError_t {
        hipError_t e = hipSuccess;
        if (p) e = hipFree(p);
        p = nullptr;
        n = 0;
        return e;
    };
    for (uint32_t w = 0; w < kMaxWs; ++w) {
        void *sp = sc->slots[w];
        RT_HIP(drop(sp, sc->slots_bytes[w]));
        sc->slots[w] = nullptr;
        RT_HIP(drop(sc->deep[w], sc->deep_bytes[w]));
        sc->deep_clean[w] = 0;
        sc->deep_meet_at[w] = 0;
    }
    void *ap = sc->acc;
    RT_HIP(drop(ap, sc->acc_bytes));
    sc->acc = nullptr;
    RT_HIP(drop(sc->wq, sc->wq_bytes));
    return RT_OK;
}
} // namespace

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
    // 64-pixel tiles (one wave's lanes for one sample), 8 x 8 (the kernel's decomposition takes
    // 2^lw x 64/2^lw; 16x4, 32x2 and 64x1 measured alike or slower for strided row shares:
    // 8-way share 0.61-0.62 ms at 8x8, 0.62 at 32x2, 0.66 at 64x1)
    k.tile_lw = 3u;
    const uint32_t tw = 1u << k.tile_lw, th = 64u >> k.tile_lw;
    const bool tiled = (P.width % tw) == 0u;
    k.tiles_x = tiled ? P.width / tw : 1u;
    k.tiled_rows = tiled ? (k.num_rows / th) * th : 0u;
    k.n_spheres = sc->n_spheres;
    k.n_materials = sc->n_materials;


    // Variant: exact (bit-exact) or fast (tolerance); clustered culling unless brute force is
    // asked for; the scalar-cache A/B variant is brute force only. Each needs its blob in LDS
    // next to the static LDS of the kernel of its traversal (sc->static_lds[culled]).
    const rt_options &O = sc->opt;
    int variant = (P.flags & RT_FLAG_FAST_MATH) ? rt::V_FAST_LDS : rt::V_EXACT_LDS;
    bool cull = !(P.flags & RT_FLAG_BRUTE_FORCE) && sc->n_clusters[1] > 0;
    const bool wave = (P.flags & RT_FLAG_WAVEFRONT) != 0u;
    if (wave && (P.flags & (RT_FLAG_FAST_MATH | RT_FLAG_SCALAR_SCENE)))
        return fail(RT_ERR_UNSUPPORTED, "rt_render_device: the wavefront variant is the exact kernel only");
    if (P.flags & RT_FLAG_SCALAR_SCENE) { variant = rt::V_EXACT_SCALAR; cull = false; }
    if (variant != rt::V_EXACT_SCALAR && static_cast<size_t>(sc->shade_offset[cull]) * 16u + sc->static_lds[cull] > sc->max_lds) {
        if (variant == rt::V_FAST_LDS || cull) return fail(RT_ERR_UNSUPPORTED, "rt_render_device: scene too large for LDS");
        variant = rt::V_EXACT_SCALAR;
    }
    if (wave && variant != rt::V_EXACT_LDS)
        return fail(RT_ERR_UNSUPPORTED, "rt_render_device: the wavefront variant needs the scene in LDS");
    if (variant == rt::V_EXACT_LDS && (O.diag & RT_DIAG_STATS) && !wave) {
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
    k.use_root = (O.diag & RT_DIAG_NO_ROOT_BOX) ? 0u : 1u;
    k.iso = (O.diag & RT_DIAG_NO_SHORTCUT) ? 0u : 1u;
    k.transpose_max = O.transpose_max;
    k.diag_unbounded_nb = (O.diag & RT_DIAG_UNBOUNDED_NB) ? 1u : 0u;
    k.fast_roots = sc->in_fast_range && camera_in_fast_range(*camera) && !(O.diag & RT_DIAG_IEEE_ROOTS) ? 1u : 0u;
    k.shade_offset = sc->shade_offset[b];
    // the shading records (the blob's tail) join the geometry in LDS unless that costs
    // workgroups per CU; RT_DIAG_SHADE_LDS / RT_DIAG_SHADE_GLOBAL force the choice (same bits)
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
    const bool shade_fits = static_cast<size_t>(k.blob_units) * 16u + sc->static_lds[cull] <= sc->max_lds;
    k.shade_lds = variant != rt::V_EXACT_SCALAR && shade_fits &&
                  ((O.diag & RT_DIAG_SHADE_LDS) ? true : (O.diag & RT_DIAG_SHADE_GLOBAL) ? false : occ_all >= occ_geo);
    k.lds_units = variant == rt::V_EXACT_SCALAR ? 0u : (k.shade_lds ? k.blob_units : k.shade_offset);
    const size_t lds = static_cast<size_t>(k.lds_units) * 16u;
    const int occ = k.shade_lds ? occ_all : occ_geo;

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
    const uint32_t deep_split = deep_off ? 0u : O.deep_split;
    // culled scenes only: with a handful of spheres (the simple scene, brute force) a deep
    // segment is cheap and the deep launch's overhead outweighs the drain it saves
    // (config 2: 0.98-1.00 vs 0.98-0.99 ms per frame)
    const bool may_split = deep_split && !wave && cull_mode == 7 && deep_split < P.max_depth;

    // Pass planning. The slot workspace of one pass (12 B per sample and pixel) stays within
    // max_pass_bytes; passes hold a multiple of 4 samples so no reduce block straddles two.
    // Frames in flight: render pass p runs on internal stream xs[p % bufs] with workspace
    // w = p % n_ws, ordered after that stream's previous render and after the caller-stream
    // work that last read workspace w (the accumulation of pass p - n_ws); render kernels
    // touch no caller memory, so the caller stream sees the same results in the same order.
    // One stream: everything on the caller stream. Under max_workspace_bytes one workspace per
    // stream goes first, then the passes shrink (frames in flight are what keeps the machine
    // full), then the streams; the bits never depend on the cut. Config 3 under 4 GiB: 2.68 ms
    // per frame in that order (7 workspaces, 52-sample passes) vs 2.79 shrinking the passes first
    // (14 workspaces, 24-sample passes), 2.56 uncapped (19.1 GiB; profiles/r04).
    const uint64_t per_sample = n_pixels * 12ull;
    // Sample pairs: a pass's full blocks of 4 samples take two pair slots each,
    // its tail samples one: half the slot memory. Their bookkeeping costs the main launch ~3% of
    // the frame period (profiles/r05/ab/pairs_cost.txt), so they are taken under a workspace cap
    // (after one workspace per stream, before shorter passes) or on request (diag `pairs`), by
    // passes issued while other renders run; a pass issued alone (a lone frame) takes single
    // samples, whose shorter items end the launch sooner (config 3: 3.23-3.26 vs 3.38-3.45 ms),
    // in a workspace of its own beside the ring. Culled LDS kernels only (the wavefront variant,
    // brute force and the scalar-cache variant store single samples).
    const bool pairs_ok = !wave && cull_mode == 7 && variant != rt::V_EXACT_SCALAR && !(O.diag & RT_DIAG_NO_PAIRS) &&
                          lds + sc->static_lds_pairs <= sc->max_lds;
    // passes dealt by tile classes: the culled LDS kernels with a scene geometry to classify
    const bool order_ok = sc->has_geom && cull_mode == 7 && !wave && variant != rt::V_EXACT_SCALAR &&
                          !(O.diag & RT_DIAG_NATURAL_ORDER);
    // the pair instantiation's own occupancy (its parked colours add static LDS): the
    // grid of a paired pass is sized by it
    int occ_pr = occ;
    if (pairs_ok) {
        int &o = sc->occ_pairs[variant][k.shade_lds ? 1 : 0];
        if (o < 0) {
            RT_HIP(rt::occupancy_render(variant, cull_mode, &o, lds, true));
            o = std::max(o, 1);
        }
        occ_pr = o;
    }
    bool pairs = pairs_ok && (O.diag & RT_DIAG_PAIRS);
    const uint32_t full_blocks_end = P.spp & ~3u;  // samples [0, full_blocks_end) form blocks of 4
    auto slot_rows = [&](uint64_t a, uint64_t b, bool pr) -> uint64_t {  // samples [a, b), a a multiple of 4
        const uint64_t nb = (std::min<uint64_t>(b, full_blocks_end) - std::min<uint64_t>(a, full_blocks_end)) / 4u;
        return pr ? (b - a) - 2u * nb : (b - a);
    };
    // the most slot rows of a pass of at most sp samples: a pass holding the tail (single samples)
    // can take more rows than a full one (pairs)
    auto max_rows = [&](uint64_t sp, bool pr) {
        uint64_t m = 0;
        for (uint64_t a = 0; a < P.spp; a += sp) m = std::max(m, slot_rows(a, std::min<uint64_t>(P.spp, a + sp), pr));
        return m;
    };
    auto ws_bytes = [&](uint64_t sp, bool pr) { return per_sample * max_rows(sp, pr); };
    const uint64_t items_cap = ((1ull << 31) - 8192) / n_pixels;  // items fit 31 bits
    uint64_t spp_full = std::min<uint64_t>({P.spp, O.max_pass_bytes / per_sample, items_cap});
    if (spp_full < P.spp) spp_full &= ~3ull;
    if (spp_full == 0) spp_full = 4;
    if (n_pixels * std::min<uint64_t>(spp_full, P.spp) >= (1ull << 31) - 8192)
        return fail(RT_ERR_INVALID, "rt_render_device: too many pixels in one call");
    auto wave_cap = [&](uint64_t sp) {
        return static_cast<uint32_t>(std::min<uint64_t>(n_pixels * std::min<uint64_t>(sp, P.spp), O.wave_queue_rays));
    };
    auto n_ws_of = [](uint32_t streams, uint32_t wsps) { return streams > 1 ? streams * wsps : 1u; };
    // Ring passes (rt_options.ring_pass_bytes): with frames in flight, a pass issued while other
    // renders run holds at most that many slot bytes, the frame's samples cut into equal passes
    // of a multiple of 4; a frame that fits one pass of max_pass_bytes and is issued alone (a
    // lone frame, the drop-in's synchronous call) still runs in one pass, in a workspace of its
    // own. The ring's 14 workspaces then hold 32-sample passes on config 3 (6.2 GiB in all
    // instead of 19.2, frame period alike: profiles/r05/ab/ring_pass.txt) and the lone frame
    // keeps its single launch pair. Ring passes hold at least kRingMinSamples samples per pixel:
    // every pass reads and writes the frame's running sums (24 B per pixel), which 4-sample
    // passes made 5% of config 4's frame (46.6 vs 44.2 ms); below that the passes stay as they were.
    constexpr uint64_t kRingMinSamples = 32;
    auto ring_of = [&](uint64_t sp, uint32_t streams) -> uint64_t {
        const uint64_t sf = std::min<uint64_t>(sp, P.spp);
        if (streams <= 1 || !O.ring_pass_bytes) return sf;
        const uint64_t cap = (O.ring_pass_bytes / per_sample) & ~3ull;
        if (cap >= sf || cap < kRingMinSamples) return sf;
        const uint64_t n = (P.spp + cap - 1) / cap;  // passes of the frame at that size
        return std::min<uint64_t>(cap, (((P.spp + n - 1) / n) + 3u) & ~3ull);
    };
    // a lone frame's one pass in its own workspace (beside the ring's smaller ones)
    auto lone_whole = [&](uint64_t sp, uint32_t streams) { return streams > 1 && sp >= P.spp && ring_of(sp, streams) < P.spp; };
    auto dq_of = [&](uint64_t sp) -> uint64_t {
        return may_split ? deep_queue_bytes(n_pixels, n_pixels * std::min<uint64_t>(sp, P.spp)) : 0u;
    };
    // the ring's workspaces (pairs when there is a ring) and the lone passes' own one (singles:
    // a whole lone frame, or a ring pass issued alone when the ring holds pairs)
    auto footprint = [&](uint32_t streams, uint32_t wsps, uint64_t sp) -> uint64_t {
        const uint64_t sr = ring_of(sp, streams);
        const bool ring_pairs = pairs && streams > 1, whole = lone_whole(sp, streams);
        uint64_t t = static_cast<uint64_t>(n_ws_of(streams, wsps)) * (ws_bytes(sr, ring_pairs) + dq_of(sr));
        if (whole) t += ws_bytes(sp, false) + dq_of(sp);
        else if (ring_pairs) t += ws_bytes(sr, false) + dq_of(sr);
        if (sr < P.spp) t += per_sample;  // the multi-pass sums
        if (wave) t += 2ull * wave_cap(sp) * 52u + 512u;
        return t;
    };
    uint32_t bufs = wave ? 1u : render_streams_of(O);  // the wavefront variant: caller stream only
    uint32_t wsps = O.workspaces_per_stream;
    uint64_t spp_pass = spp_full;
    if (const uint64_t cap = O.max_workspace_bytes) {
        while (footprint(bufs, wsps, spp_pass) > cap) {
            if (bufs > 1 && wsps > 1) {
                wsps = 1;
                continue;
            }
            if (bufs > 1 && pairs_ok && !pairs) {
                pairs = true;
                continue;
            }
            if (spp_pass > 4) {
                spp_pass = std::max<uint64_t>(4, (std::min<uint64_t>(spp_pass, P.spp) - 1) & ~3ull);
                continue;
            }
            spp_pass = spp_full;
            if (bufs > 1) --bufs;
            else return fail(RT_ERR_CAPACITY, "rt_render_device: max_workspace_bytes " + std::to_string(cap) +
                                                  " below one 4-sample pass of this frame (" +
                                                  std::to_string(footprint(1, 1, 4)) + " bytes)");
        }
    }
    const bool pipe = bufs > 1;
    const uint32_t n_ws = n_ws_of(bufs, wsps);
    const uint64_t spe = std::min<uint64_t>(spp_pass, P.spp);  // a lone pass
    const uint64_t spr = ring_of(spp_pass, bufs);                // a ring pass
    const bool ring_pairs = pairs && pipe, whole = lone_whole(spp_pass, bufs);
    const uint32_t lone_ws = (ring_pairs || whole) ? n_ws : kMaxWs;  // the lone passes' workspace (singles), if any
    auto pass_of = [&](uint32_t w) { return w == lone_ws && whole ? spe : spr; };
    auto ws_size = [&](uint32_t w) { return ws_bytes(pass_of(w), ring_pairs && w != lone_ws); };
    // under a cap, workspaces left larger (or more numerous) by earlier frames are re-cut once
    if (O.max_workspace_bytes) {
        uint64_t after = 0;
        for (uint32_t w = 0; w < kMaxWs; ++w) {
            const bool used = w < n_ws || w == lone_ws;
            after += used ? std::max<uint64_t>(sc->slots_bytes[w], ws_size(w)) : sc->slots_bytes[w];
            after += used && may_split ? std::max<uint64_t>(sc->deep_bytes[w], dq_of(pass_of(w))) : sc->deep_bytes[w];
        }
        after += spr < P.spp ? std::max<uint64_t>(sc->acc_bytes, per_sample) : sc->acc_bytes;
        after += wave ? std::max<uint64_t>(sc->wq_bytes, 2ull * wave_cap(spp_pass) * 52u + 512u) : sc->wq_bytes;
        if (after > O.max_workspace_bytes)
            if (int rc = free_workspaces(sc); rc) return rc;
    }
    sc->used_streams = bufs;
    sc->used_ws = n_ws + (lone_ws < kMaxWs ? 1u : 0u);
    sc->used_pass = static_cast<uint32_t>(spr);
    sc->used_deep = 0;
    sc->used_pairs = sc->used_split = sc->used_lead = sc->used_sky = 0;
    if (spr < P.spp)
        if (int rc = ensure((void **)&sc->acc, &sc->acc_bytes, per_sample); rc) return rc;
    for (uint32_t w = 0; w < n_ws; ++w)
        if (int rc = ensure((void **)&sc->slots[w], &sc->slots_bytes[w], ws_size(w)); rc) return rc;
    if (lone_ws < kMaxWs)
        if (int rc = ensure((void **)&sc->slots[lone_ws], &sc->slots_bytes[lone_ws], ws_size(lone_ws)); rc) return rc;
    // wavefront variant: two ray queues of cap rays (52 B each) and their counters
    uint32_t wcap = 0;
    rt::RayQueue wqa{}, wqb{};
    int wgrid = 0;
    if (wave) {
        wcap = wave_cap(spp_pass);
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

    // the frame's dealing order (not with sample pairs) and the sky kernel: the
    // tiles proven to send every primary ray to the sky are rendered by sky_kernel at the frame's
    // last pass (all samples, one thread per pixel, no slots), the passes deal the others
    const rt_scene::Order *ord = nullptr;
    if (order_ok && !pairs)
        if (int rc = pass_order(sc, *camera, k, &ord); rc) return rc;
    // (max_depth 0: every sample's colour is 0, main.cxx:74, not the sky's)
    const bool sky_kernel = ord && ord->d_perm && ord->t.n_sky && P.max_depth > 0 && !(O.diag & RT_DIAG_NO_SKY);
    const uint32_t sky_pos0 = sky_kernel ? static_cast<uint32_t>(64u * (ord->t.perm.size() - ord->t.n_sky)) : k.n_pixels;
    const uint32_t ring = static_cast<uint32_t>(sc->calls % rt_scene::kRing);
    ++sc->calls;
    auto others_running = [&] { return pipe && sc->last_ws >= 0 && hipEventQuery(sc->ev_done[sc->last_ws]) == hipErrorNotReady; };
    // a frame issued alone that fits one pass takes it whole (lone_whole); otherwise ring passes
    const uint64_t first_pass = whole && !others_running() && !(O.diag & RT_DIAG_IN_FLIGHT) ? spe : spr;
    for (uint32_t s0 = 0, s1 = 0; s0 < P.spp; s0 = s1) {
        s1 = static_cast<uint32_t>(std::min<uint64_t>(P.spp, s0 + (s0 == 0 ? first_pass : spr)));
        // another render still running? (then this one takes a partial grid, grid_wg_per_cu)
        const bool in_flight = others_running() || (pipe && (O.diag & RT_DIAG_IN_FLIGHT));
        // every pass takes the next workspace and stream: pass p + 1's render overlaps pass
        // p's drain and accumulation, within a frame and across frames; a whole lone frame, and
        // a pass issued alone when the ring holds pairs, take the lone passes' workspace (single
        // samples)
        const bool pass_pairs = ring_pairs && in_flight;
        uint32_t wb = 0;
        if (lone_ws < kMaxWs && ((s1 - s0) > spr || (ring_pairs && !in_flight))) {
            wb = lone_ws;
        } else if (pipe) {
            wb = sc->next_buf % n_ws;
            sc->next_buf = wb + 1u;
        }
        hipStream_t xst = pipe ? sc->xs[wb % bufs] : st;
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
        k.n_pair_items = static_cast<uint32_t>(((s1 - s0) - slot_rows(s0, s1, pass_pairs)) * n_pixels);
        if (k.n_pair_items) ++sc->used_pairs;
        // dealing order: lead tiles first, then the others (then the proven sky
        // tiles, unless the sky kernel renders them) in single-sample passes of the culled LDS
        // kernels, else the natural order
        const bool ordered = ord && ord->d_perm && !k.n_pair_items;
        fill_frame_consts(k);
        // items: the pass's pair items and its single tail samples (one slot each); with the sky
        // kernel, the positions before the sky tiles'
        const uint64_t n_samples = n_pixels * (s1 - s0);
        k.n_items = static_cast<uint32_t>((ordered && sky_kernel ? sky_pos0 : n_pixels) * slot_rows(s0, s1, pass_pairs));
        k.n_slots = static_cast<uint32_t>(n_pixels * slot_rows(s0, s1, pass_pairs));
        int wg_cu = grid_wg_per_cu(pass_pairs ? occ_pr : occ, in_flight, bufs, n_samples);
        // A lone pass whose sky kernel runs beside it: the main launch's workgroups fill every
        // CU's registers (72 VGPRs x 7 waves per SIMD), so the sky kernel would start only as they
        // retire and end the frame after them. The main launch leaves room in proportion to the
        // sky's share of the pixels (config 3, 73% sky: 2 of 7 workgroups per CU; lone frame
        // 2.466-2.474 ms vs 2.528-2.547 with none, 2.474-2.495 with 1; period unchanged;
        // profiles/r06/ab/sky_room.txt). RT_LONE_SKY_ROOM >= 0 (A/B build switch) fixes it.
        if (!in_flight && sky_kernel && ordered && s1 == P.spp && pipe && !(O.diag & RT_DIAG_SKY_SERIAL)) {
            const double sky_frac = 1.0 - static_cast<double>(sky_pos0) / static_cast<double>(n_pixels);
            const int room = RT_LONE_SKY_ROOM >= 0 ? RT_LONE_SKY_ROOM : static_cast<int>(wg_cu * sky_frac * 0.4 + 0.5);
            wg_cu = std::max(1, wg_cu - room);
        }
        const uint32_t grid = static_cast<uint32_t>(
            std::max<uint64_t>(1, std::min<uint64_t>(static_cast<uint64_t>(wg_cu) * sc->cu_count, (k.n_items + 255u) / 256u)));
        k.n_blocks = (k.n_items + 63u) / 64u;
        k.guided_l2b = guided_l2b(grid * 4u, in_flight);
        k.block_perm = nullptr;
        k.n_groups = 1;
        k.grp_blocks[0] = k.n_blocks;
        k.grp_items[0] = k.n_items;
        k.grp_pix[0] = 0;
        k.grp_pix[1] = k.grp_pix[2] = k.grp_pix[3] = k.n_pixels;
        k.div_grp[0] = make_udiv(k.n_pixels);
        if (ordered) {
            const rthost::tile_order &t = ord->t;
            const uint64_t S = s1 - s0;
            const uint64_t nbl[3] = {t.n_lead, t.perm.size() - t.n_lead - t.n_sky, sky_kernel ? 0u : t.n_sky};
            k.block_perm = ord->d_perm;
#ifdef RT_ORDER_NULLPERM  // A/B build switch (with RT_ORDER_IDENTITY): the identity permutation not read
            k.block_perm = nullptr;
#endif
            k.n_groups = sky_kernel ? 2 : 3;
            for (int g = 0; g < 3; ++g) {
                k.grp_pix[g + 1] = k.grp_pix[g] + static_cast<uint32_t>(64u * nbl[g]);
                k.grp_items[g] = static_cast<uint32_t>(64u * nbl[g] * S);
                k.grp_blocks[g] = static_cast<uint32_t>(nbl[g] * S);  // nbl[g] blocks per sample
                k.div_grp[g] = make_udiv(static_cast<uint32_t>(std::max<uint64_t>(64u * nbl[g], 1u)));
            }
            sc->used_lead = t.n_lead;
            sc->used_sky = sky_kernel ? t.n_sky : 0u;
        } else {
            sc->used_lead = sc->used_sky = 0;
        }
        // deep-path split: this workspace's deep queue (its counters in the queue-counter block)
        k.deep_depth = 0;
        k.deep_mode = 0;
        bool two_part = false;
        uint32_t stats_waves = 0;  // the instrumented build: waves of the launch the counters cover
        // (diag lone_unsplit: a lone pass dealt by tile classes is not split, its trapped paths
        // starting in its first items; slower, the accumulation then waits for the whole launch)
        if (may_split && (n_samples >= O.deep_min_items || in_flight) &&
            (in_flight || !ordered || !(O.diag & RT_DIAG_LONE_UNSPLIT))) {
            const uint32_t rcap = deep_region_cap(n_samples), cap = 8u * rcap;
            const size_t px_bytes = deep_px_bytes(n_pixels);
            bool fresh = false;
            if (int rc = ensure(&sc->deep[wb], &sc->deep_bytes[wb], deep_queue_bytes(n_pixels, n_samples), &fresh); rc)
                return rc;
            if (fresh) {  // new memory: no flag set, no pair arrival counted
                sc->deep_clean[wb] = 0;
                RT_HIP(hipMemsetAsync(sc->deep[wb], 0, sc->deep_bytes[wb], xst));
            } else if (sc->deep_meet_at[wb] != px_bytes + static_cast<size_t>(cap) * 56u) {
                // another layout: its arrival words lie where other arrays were (every pass that
                // keeps the layout leaves them zero: the second arrival of a pair resets its word)
                RT_HIP(hipMemsetAsync(static_cast<char *>(sc->deep[wb]) + px_bytes + static_cast<size_t>(cap) * 56u, 0,
                                      static_cast<size_t>(cap) * 4u, xst));
            }
            sc->deep_meet_at[wb] = px_bytes + static_cast<size_t>(cap) * 56u;
            if (sc->deep_clean[wb] < px_bytes)  // flags over bytes a queue may have used
                RT_HIP(hipMemsetAsync(sc->deep[wb], 0, px_bytes, xst));
            // every accumulation clears the flags its pass set, and the bytes past px_bytes are
            // this pass's queue storage: only the leading px_bytes are known to be zero after it
            sc->deep_clean[wb] = px_bytes;
            char *base = static_cast<char *>(sc->deep[wb]);
            k.deep.px = reinterpret_cast<uint8_t *>(base);
            base += px_bytes;
            k.deep.f = reinterpret_cast<float *>(base);
            k.deep.rng = reinterpret_cast<uint64_t *>(base + static_cast<size_t>(cap) * 36u);
            k.deep.slot = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(cap) * 44u);
            k.deep.hid = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(cap) * 48u);
            k.deep.link = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(cap) * 52u);
            k.deep.meet = reinterpret_cast<uint32_t *>(base + static_cast<size_t>(cap) * 56u);
            k.deep.ctr = k.queue_ctr;
            k.deep.rcap = rcap;
            k.deep_depth = deep_split;
            two_part = RT_TWO_PART && pipe && !in_flight;
        }
        if (O.diag & RT_DIAG_VERBOSE)
            std::fprintf(stderr, "[rt] variant=%d cull=%d shade_lds=%u lds=%zu B occ=%d WG/CU cus=%d grid=%u items=%u "
                                 "samples=[%u,%u) streams=%u workspaces=%u split=%u guided log2(beta)*1e6=%u\n",
                         variant, cull_mode, k.shade_lds, lds, occ, sc->cu_count, grid, k.n_items, s0, s1, bufs, n_ws,
                         k.deep_depth, static_cast<uint32_t>(-k.guided_l2b * 1e6f));
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
            stats_waves = grid * 4u;
            if (two_part) {
                if (!sc->ev_main[wb]) RT_HIP(hipEventCreateWithFlags(&sc->ev_main[wb], hipEventDisableTiming));
                RT_HIP(hipEventRecord(sc->ev_main[wb], xst));
            }
            if (k.deep_depth) {  // the deep launch: the queued paths, same grid, same stream
                ++sc->used_split;
                rt::KParams kd = k;
                kd.deep_mode = k.deep_depth;
                kd.deep_depth = 0;
                // the deep paths bounce inside glass spheres, inside the box over all clusters:
                // the level-3 gate only costs there (alike within box noise, fewer box tests;
                // same bits)
                kd.use_root = 0u;
#ifdef RT_DEEP_TMAX  // A/B build switch: every deep launch's transposition threshold
                kd.transpose_max = std::min<uint32_t>(O.transpose_max, RT_DEEP_TMAX);
#endif
                // its waves at the top issue priority: each path is a chain of ~56 dependent
                // iterations, and beside other renders' waves every iteration waits for the
                // SIMD's other waves (config 3's 8-way share, split, 7 streams: 0.513-0.515 ms vs
                // 0.569-0.571; profiles/r03/ab/deep_prio.txt)
                kd.deep_prio = 1u;
                // the shading records in LDS for the deep launch of a pass issued alone: its
                // paths bounce in glass and shade every segment, and its few busy waves wait on
                // each global round trip (config 3 single frame: deep launch 0.59 vs 0.65 ms).
                // Not beside other renders: its larger workgroups then displace theirs (frame
                // stream 2.69-2.73 vs 2.57-2.59 ms per frame, 8-way share 0.45 vs 0.42)
                int wpb = 4;
                uint32_t dgrid = grid;
                if (RT_DEEP_LDS_STAGE && !in_flight && variant != rt::V_EXACT_SCALAR && !k.shade_lds && shade_fits) {
                    kd.shade_lds = 1u;
                    kd.lds_units = k.blob_units;
                    // 8-wave groups share the LDS copy (3 x 8 waves per CU instead of 3 x 4), the
                    // grid is what is resident at once, and the chunks are dealt statically: the
                    // launch was ~0.28 ms even for paths of one segment, most of it thousands of
                    // waves probing the regions' counters and groups waiting for residency
                    int &ow = sc->occ_deep_wide[variant];
                    if (ow < 0) {
                        const size_t bytes = static_cast<size_t>(k.blob_units) * 16u;
                        size_t st8 = 0, st4 = 0;
                        int o8 = 0, o4 = 0;
                        RT_HIP(rt::deep_occupancy(variant, 8, bytes, &o8, &st8));
                        // against the 4-wave deep kernel it replaces, with the same blob in LDS
                        // (the main kernel's occupancy stood in for it)
                        RT_HIP(rt::deep_occupancy(variant, 4, bytes, &o4, &st4));
                        // (the instrumented kernel follows the product's choice: wide whenever it fits)
                        ow = bytes + st8 <= sc->max_lds && (o8 * 8 > o4 * 4 || (variant == rt::V_STATS_LDS && o8 > 0)) ? o8 : 0;
                    }
                    if (RT_DEEP_WIDE && ow > 0) {
                        wpb = 8;
                        dgrid = static_cast<uint32_t>(ow * sc->cu_count);
                        kd.deep_static = RT_DEEP_STATIC ? 1u : 0u;
                        // its waves run alone on their SIMDs, so a cluster's transposed member
                        // test (three LDS round trips) pays off for fewer requesting lanes: at
                        // most 4 here (lone deep launch 0.351-0.360 vs 0.370-0.377 ms at 16;
                        // 1-8 alike, per-lane tests always 0.400-0.405; profiles/r05/deep/
                        // lone_deep_tmax.txt)
                        kd.transpose_max = std::min<uint32_t>(O.transpose_max, RT_LONE_DEEP_TMAX);
                    }
                }
                if (variant == rt::V_STATS_LDS && (O.diag & RT_DIAG_STATS_DEEP_ONLY)) {
                    // diagnostics: the counters and events of the deep launch alone
                    RT_HIP(hipMemsetAsync(sc->dbg, 0, 16 * sizeof(unsigned long long), xst));
                    RT_HIP(hipMemsetAsync(sc->dbg + rt::kDbgEvBase, 0, rt::kDbgEvents * sizeof(unsigned long long), xst));
                }
                RT_HIP(rt::launch_render(variant, cull_mode, kd, dgrid, xst, wpb));
                sc->used_deep = static_cast<uint32_t>(wpb) | (kd.deep_static ? 16u : 0u);
                if (variant == rt::V_STATS_LDS && (O.diag & RT_DIAG_STATS_DEEP_ONLY)) stats_waves = dgrid * static_cast<uint32_t>(wpb);
            }
        }
        bool sky_aside = false;  // the sky kernel on another stream (then the accumulation waits for ev_sky)
        if (sky_kernel && s1 == P.spp) {
            // the sky tiles' pixels, every sample of the frame; position i's sum to its sample-0
            // slot (which no pass of these groups uses), read by this pass's accumulation. A pass
            // issued alone runs it on another stream, after the workspace is free, beside the main
            // launch (which leaves it room) and the deep launch; beside other renders it follows
            // the pass on its stream
            rt::KSky ks{};
            ks.fc = k.fc;
            ks.block_perm = k.block_perm;
            ks.pos0 = sky_pos0;
            ks.n_pix = k.n_pixels - sky_pos0;
            ks.sums = k.slots + 3u * static_cast<size_t>(sky_pos0);
            ks.segments = k.segments;
            sky_aside = pipe && !in_flight && !(O.diag & RT_DIAG_SKY_SERIAL);
            if (sky_aside) {
                // the next render stream, not a stream of its own: HIP maps streams to hardware
                // queues round-robin in creation order, and a ninth stream shared a queue with one
                // of the render streams, behind whose main launch the sky kernel then waited (one
                // lone frame in three at 4 queues: 0.83 vs 0.69 ms on the 8-way share). Consecutive
                // render streams sit on different queues.
                hipStream_t sky_st = sc->xs[(wb % bufs + 1u) % bufs];
                if (sc->free_valid[wb]) RT_HIP(hipStreamWaitEvent(sky_st, sc->ev_free[wb], 0));
                // (the counters it adds to are this pass's: zeroed on xst before the main launch)
                if (ks.segments) {
                    if (!sc->ev_main[wb]) RT_HIP(hipEventCreateWithFlags(&sc->ev_main[wb], hipEventDisableTiming));
                    if (!two_part) RT_HIP(hipEventRecord(sc->ev_main[wb], xst));
                    RT_HIP(hipStreamWaitEvent(sky_st, sc->ev_main[wb], 0));
                }
                RT_HIP(rt::launch_sky(ks, sky_st));
                RT_HIP(hipEventRecord(sc->ev_sky, sky_st));
            } else {
                RT_HIP(rt::launch_sky(ks, xst));
            }
        }
        if (variant == rt::V_STATS_LDS) sc->dbg_waves = stats_waves;
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
        a.paired = k.n_pair_items ? 1u : 0u;
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
        a.block_perm = k.block_perm;
        a.sky_pos0 = sky_pos0;
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
        if (sky_aside) RT_HIP(hipStreamWaitEvent(st, sc->ev_sky, 0));
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

int rt_scene_usage_get(const rt_scene *sc, rt_scene_usage *out)
{
    if (!sc || !out) return fail(RT_ERR_INVALID, "rt_scene_usage_get: null argument");
    rt_scene_usage u{};
    uint64_t ws = sc->acc_bytes + sc->wq_bytes;
    for (uint32_t w = 0; w < kMaxWs; ++w) ws += sc->slots_bytes[w] + sc->deep_bytes[w];
    uint64_t fixed = kCtrWords * sizeof(uint32_t) + (sc->dbg ? rt::kDbgWords * sizeof(unsigned long long) : 0u);
    for (int b = 0; b < 2; ++b) fixed += static_cast<uint64_t>(sc->blob_units[b]) * 16u;
    u.device_bytes = ws + fixed;
    u.workspace_bytes = ws;
    u.render_streams = sc->used_streams;
    u.workspaces = sc->used_ws;
    u.pass_samples = sc->used_pass;
    u.deep_launch = sc->used_deep;
    u.pair_passes = sc->used_pairs;
    u.split_passes = sc->used_split;
    u.lead_tiles = sc->used_lead;
    u.sky_tiles = sc->used_sky;
    u.static_lds_bytes = static_cast<uint32_t>(sc->static_lds[1]);
    u.max_lds_bytes = static_cast<uint32_t>(sc->max_lds);
    *out = u;
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
    // the instrumented kernel's bounds check (rt_device.h kDbgError): an index past its bound
    if (const uint64_t e = out[rt::kDbgError]; e) {
        static const char *const kWhat[] = {"?", "walk-shortcut neighbour slot", "shading record", "sample slot",
                                            "deep-queue append", "deep-queue item", "deep-path hint sphere", "cluster members",
                                            "deep pixel flag"};
        const uint32_t code = static_cast<uint32_t>(e >> 32);
        return fail(RT_ERR_DEVICE, std::string("rt_scene_debug_counters: bounds check: ") +
                                       kWhat[code < sizeof(kWhat) / sizeof(kWhat[0]) ? code : 0] + " index " +
                                       std::to_string(static_cast<uint32_t>(e)) + " past its bound (code " +
                                       std::to_string(code) + ")");
    }
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

// The synchronous renders' per-device context, kept between calls: the reference's entry point
// (cuda_impl, src/CUDA/cuda_impl.cu:384-453) is called once per frame with the same scene, and
// building the scene (clusters, shortcut words, streams, events), its workspaces and the frame
// buffers on every call cost more than the frame itself. The context is keyed by the scene's
// records and the options its scene would be created with (rt_get_default_options at the call):
// another scene or other options rebuild it. rt_release_cached frees it.
struct SyncContext {
    std::vector<unsigned char> key;
    rt_scene *sc = nullptr;
    float *d_rgb = nullptr;
    size_t rgb_bytes = 0;
    uint8_t *d_u8 = nullptr;
    size_t u8_bytes = 0;
    uint64_t *d_seg = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
};
std::mutex g_sync_mu;  // one synchronous render at a time per process (the reference's entry is not re-entrant)
std::map<int, SyncContext> g_sync;

void sync_release(int dev, SyncContext &c)
{
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(dev);
    if (c.sc) rt_scene_destroy(c.sc);
    for (void *p : {(void *)c.d_rgb, (void *)c.d_u8, (void *)c.d_seg})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : {c.e0, c.e1})
        if (e) (void)hipEventDestroy(e);
    c = SyncContext{};
    (void)hipSetDevice(prev);
}

// Synchronous host-buffer render on the current device (the cuda_impl replacement).
int render_host(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                const rt_camera *camera, const rt_params *params, float *rgb_out, uint8_t *u8_out, rt_stats *stats)
{
    if (!camera || (!rgb_out && !u8_out)) return fail(RT_ERR_INVALID, "render: null argument");
    if (int rc = check_params(params); rc != RT_OK) return rc;
    if ((n_spheres && !spheres) || !materials || !n_materials) return fail(RT_ERR_INVALID, "render: null scene");
    const auto t0 = std::chrono::steady_clock::now();
    int dev = 0;
    RT_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(g_sync_mu);
    SyncContext &cx = g_sync[dev];
    {
        rt_options opt;
        if (int rc = rt_get_default_options(&opt); rc) return rc;
        std::vector<unsigned char> key(sizeof(rt_sphere) * n_spheres + sizeof(rt_material) * n_materials + sizeof(opt));
        unsigned char *k = key.data();
        if (n_spheres) std::memcpy(k, spheres, sizeof(rt_sphere) * n_spheres);
        k += sizeof(rt_sphere) * n_spheres;
        std::memcpy(k, materials, sizeof(rt_material) * n_materials);
        k += sizeof(rt_material) * n_materials;
        std::memcpy(k, &opt, sizeof(opt));
        if (!cx.sc || key != cx.key) {
            sync_release(dev, cx);
            if (int rc = rt_scene_create(spheres, n_spheres, materials, n_materials, dev, &cx.sc); rc) return rc;
            cx.key.swap(key);
        }
    }
    rt_scene *sc = cx.sc;
    const rt_params &P = *params;
    const uint64_t rows = (P.flags & RT_FLAG_FULL_FRAME) ? P.height : rows_of(P);
    const uint64_t n_values = rows * P.width * 3u;
    int rc = RT_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == RT_OK) rc = fail(RT_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
        return rc == RT_OK;
    };
    auto grow_buf = [&](void **p, size_t *have, size_t want) {
        if (*have >= want && *p) return;
        if (*p) chk(hipFree(*p), "hipFree");
        *p = nullptr;
        *have = 0;
        if (chk(hipMalloc(p, std::max<size_t>(want, 256)), "hipMalloc")) *have = want;
    };
    grow_buf((void **)&cx.d_rgb, &cx.rgb_bytes, n_values * 4);
    if (u8_out) grow_buf((void **)&cx.d_u8, &cx.u8_bytes, n_values);
    if (rc == RT_OK && !cx.d_seg) chk(hipMalloc((void **)&cx.d_seg, 24), "hipMalloc");
    if (rc == RT_OK && !cx.e0) chk(hipEventCreate(&cx.e0), "hipEventCreate");
    if (rc == RT_OK && !cx.e1) chk(hipEventCreate(&cx.e1), "hipEventCreate");
    float *d_rgb = cx.d_rgb;
    uint8_t *d_u8 = cx.d_u8;
    uint64_t *d_seg = cx.d_seg;
    hipEvent_t e0 = cx.e0, e1 = cx.e1;
    if (rc == RT_OK && (P.flags & RT_FLAG_FULL_FRAME)) chk(hipMemsetAsync(d_rgb, 0, n_values * 4, nullptr), "hipMemset");
    // the work counters (rt_stats) come from the counting instantiation of the kernels, slower than
    // the product's: only when the caller asks for them (rt::render_impl does not, as cuda_impl)
    if (rc == RT_OK && stats) chk(hipMemsetAsync(d_seg, 0, 24, nullptr), "hipMemset");
    if (rc == RT_OK) chk(hipEventRecord(e0, nullptr), "hipEventRecord");
    if (rc == RT_OK) rc = rt_render_device(sc, camera, params, d_rgb, nullptr, stats ? d_seg : nullptr);
    if (rc == RT_OK) chk(hipEventRecord(e1, nullptr), "hipEventRecord");
    if (rc == RT_OK && u8_out) rc = rt_epilogue_rgb8_device(d_rgb, d_u8, n_values / 3, nullptr);
    uint64_t segs[3] = {0, 0, 0};
    float ms = 0.f;
    // the copies on the null stream follow the render; the last one returns when all is done
    if (rc == RT_OK && rgb_out) chk(hipMemcpy(rgb_out, d_rgb, n_values * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == RT_OK && u8_out) chk(hipMemcpy(u8_out, d_u8, n_values, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == RT_OK && stats) chk(hipMemcpy(segs, d_seg, 24, hipMemcpyDeviceToHost), "hipMemcpy");
    if (rc == RT_OK) chk(hipDeviceSynchronize(), "render");
    if (rc == RT_OK) chk(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
    if (rc != RT_OK) {
        // a failed call leaves no state behind: the next one starts from a new context
        const std::string msg = g_error;
        sync_release(dev, cx);
        g_error = msg;
    }
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

int rt_release_cached(void)
{
    std::lock_guard<std::mutex> lock(g_sync_mu);
    for (auto &kv : g_sync) sync_release(kv.first, kv.second);
    g_sync.clear();
    return RT_OK;
}

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

// RT_DIAG_STANDIN_TRANSPORT: RCCL's point-to-point calls restated as stream-ordered device
// copies between ranks that share one device, so that the RCCL gather branch of
// rt_multi_render_device (grouped send/recv per peer on the ranks' streams, slot offsets, tile
// reuse across frames in flight) runs on one GPU. Semantics kept: within a group, a send on
// rank a's stream to peer b pairs with the receive on rank b's stream from a; the receive's
// stream waits for the send stream's prior work, copies, and the send stream's later work
// waits for the copy (the tile may not be overwritten before it has left), as with RCCL.
namespace standin {
struct comm { int rank, n, dev; };
struct op { bool is_send; const void *src; void *dst; size_t bytes; int peer; comm *c; hipStream_t st; };
thread_local std::vector<op> g_ops;
thread_local int g_depth = 0;
size_t type_bytes(ncclDataType_t t) { return t == ncclFloat ? 4u : t == ncclUint8 ? 1u : 0u; }
ncclResult_t comm_init_all(ncclComm_t *comms, int n, const int *devs)
{
    for (int i = 0; i < n; ++i) comms[i] = reinterpret_cast<ncclComm_t>(new comm{i, n, devs ? devs[i] : i});
    return ncclSuccess;
}
ncclResult_t comm_destroy(ncclComm_t c)
{
    delete reinterpret_cast<comm *>(c);
    return ncclSuccess;
}
ncclResult_t push(bool is_send, const void *src, void *dst, size_t count, ncclDataType_t t, int peer, ncclComm_t c,
                  hipStream_t st)
{
    comm *cc = reinterpret_cast<comm *>(c);
    if (!cc || !type_bytes(t) || peer < 0 || peer >= cc->n || peer == cc->rank) return ncclInvalidArgument;
    // only grouped calls are emulated: a call outside a group is refused and leaves nothing behind
    // for the next group to pair with
    if (!g_depth) return ncclInvalidUsage;
    g_ops.push_back({is_send, src, dst, count * type_bytes(t), peer, cc, st});
    return ncclSuccess;
}
ncclResult_t send(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t st)
{
    return push(true, buf, nullptr, count, t, peer, c, st);
}
ncclResult_t recv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t st)
{
    return push(false, nullptr, buf, count, t, peer, c, st);
}
ncclResult_t group_start()
{
    if (!g_depth) g_ops.clear();
    ++g_depth;
    return ncclSuccess;
}
ncclResult_t group_end()
{
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth) return ncclSuccess;
    std::vector<op> ops;
    ops.swap(g_ops);
    std::vector<bool> used(ops.size(), false);
    ncclResult_t res = ncclSuccess;
    for (size_t i = 0; i < ops.size() && res == ncclSuccess; ++i) {
        if (!ops[i].is_send) continue;
        const op &sd = ops[i];
        size_t j = 0;
        for (; j < ops.size(); ++j)
            if (!used[j] && !ops[j].is_send && ops[j].c->rank == sd.peer && ops[j].peer == sd.c->rank) break;
        if (j == ops.size() || ops[j].bytes != sd.bytes) {
            res = ncclInvalidUsage;
            break;
        }
        used[i] = used[j] = true;
        const op &rv = ops[j];
        hipEvent_t sent = nullptr, landed = nullptr;
        if (hipEventCreateWithFlags(&sent, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&landed, hipEventDisableTiming) != hipSuccess || hipEventRecord(sent, sd.st) != hipSuccess ||
            hipStreamWaitEvent(rv.st, sent, 0) != hipSuccess ||
            hipMemcpyAsync(rv.dst, sd.src, sd.bytes, hipMemcpyDeviceToDevice, rv.st) != hipSuccess ||
            hipEventRecord(landed, rv.st) != hipSuccess || hipStreamWaitEvent(sd.st, landed, 0) != hipSuccess)
            res = ncclUnhandledCudaError;
        if (sent) (void)hipEventDestroy(sent);
        if (landed) (void)hipEventDestroy(landed);
    }
    for (size_t i = 0; i < ops.size() && res == ncclSuccess; ++i)
        if (!used[i]) res = ncclInvalidUsage;  // a receive without its send
    return res;
}
const char *error_string(ncclResult_t r) { return r == ncclSuccess ? "success" : "stand-in transport: unmatched or failed call"; }
} // namespace standin

const rccl_api &standin_api()
{
    static rccl_api api = [] {
        rccl_api a;
        a.comm_init_all = standin::comm_init_all;
        a.comm_destroy = standin::comm_destroy;
        a.send = standin::send;
        a.recv = standin::recv;
        a.group_start = standin::group_start;
        a.group_end = standin::group_end;
        a.error_string = standin::error_string;
        a.ok = true;
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
    const rccl_api *api = nullptr;  // RCCL, or the stand-in (RT_DIAG_STANDIN_TRANSPORT)
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
    return rt_multi_create_ex(spheres, n_spheres, materials, n_materials, devices, n_ranks, nullptr, out);
}

int rt_multi_create_ex(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                       const int *devices, int n_ranks, const rt_options *options, rt_multi **out)
{
    if (!out) return fail(RT_ERR_INVALID, "rt_multi_create: null output");
    *out = nullptr;
    rt_options opt;
    if (options) {
        if (int rc = check_options(*options); rc) return rc;
        opt = *options;
    } else if (int rc = default_options(opt); rc) {
        return rc;
    }
    // two supported layouts: every rank on its own device (RCCL), or every rank on rank 0's
    // device (virtual ranks); a mix would gather through cross-device copies no test covers.
    // Checked before any HIP call.
    bool distinct = true, all_same = true;
    if (devices && n_ranks > 0) {
        if (n_ranks > 64) return fail(RT_ERR_INVALID, "rt_multi_create: at most 64 ranks");
        for (int r = 1; r < n_ranks; ++r) {
            all_same = all_same && devices[r] == devices[0];
            for (int q = 0; q < r; ++q) distinct = distinct && devices[q] != devices[r];
        }
        if (!distinct && !all_same)
            return fail(RT_ERR_INVALID, "rt_multi_create: devices must be all distinct or all rank 0's device");
    }
    const bool standin = (opt.diag & RT_DIAG_STANDIN_TRANSPORT) != 0u;
    if (standin && !(devices && n_ranks > 1 && all_same))
        return fail(RT_ERR_INVALID, "rt_multi_create: the stand-in transport needs two or more ranks on one device");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_ERR_DEVICE, "rt_multi_create: no HIP device");
    const int N = n_ranks <= 0 ? ndev : n_ranks;
    if (!devices && N > ndev) return fail(RT_ERR_INVALID, "rt_multi_create: more ranks than devices (pass a device list)");
    if (N > 64) return fail(RT_ERR_INVALID, "rt_multi_create: at most 64 ranks");
    for (int r = 0; r < N; ++r) {
        const int d = devices ? devices[r] : r;
        if (d < 0 || d >= ndev) return fail(RT_ERR_INVALID, "rt_multi_create: bad device index");
    }
    rt_multi *m = new rt_multi();
    m->n = N;
    for (int r = 0; r < N; ++r) m->dev.push_back(devices ? devices[r] : r);
    m->rccl = N > 1 && (distinct || standin);
    m->api = standin ? &standin_api() : &rccl();
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
        rc = rt_scene_create_ex(spheres, n_spheres, materials, n_materials, m->dev[r], &opt, &m->sc[r]);
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
        const rccl_api &api = *m->api;
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
        if (c) m->api->comm_destroy(c);
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
        const rccl_api &api = *m->api;
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


} // extern "C"
