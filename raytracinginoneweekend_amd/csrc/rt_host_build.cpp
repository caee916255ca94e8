// rt_host_build.cpp — host-only half of the C-ABI (include/rt_api.h): the reference's camera
// and scene constructors bit for bit, options, the scene blob (always-tested list + clusters)
// and the walk-shortcut proofs, exact-division checks, the PPM writer. No HIP here, so that the
// CPU sanitizer builds (tests/sanitize/Makefile) compile this file as it ships.
//
// Compiled with -ffp-contract=off: the camera basis and the huge-scene generator must round
// exactly like the reference's (g++, x86-64 SSE, no contraction).
#include "rt_host_build.h"

#include <algorithm>
#include <cerrno>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace rthost {

thread_local std::string g_error;

int fail(int code, const std::string &msg)
{
    g_error = msg;
    return code;
}

} // namespace rthost

using namespace rthost;

namespace {

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

} // namespace

namespace rthost {

// ---- options (include/rt_api.h rt_options) ---------------------------------------------
// The library reads two environment variables: GPU_MAX_HW_QUEUES (HIP's own, read when HIP
// starts; the render streams follow it) and RT_OPTIONS (rt_options_parse syntax, applied once
// over the defaults). Everything else that steers a render is a field of the scene's options.
rt_options library_defaults()
{
    rt_options o{};
    o.size = sizeof(rt_options);
    o.render_streams = 0;  // auto: GPU_MAX_HW_QUEUES - 1 within 2..7 (render_streams_of)
    o.workspaces_per_stream = 2;
    o.deep_split = 8;
    o.max_pass_bytes = kMaxSlotsBytes;
    o.max_workspace_bytes = 0;
    o.deep_min_items = 1ull << 25;
    o.cluster_size = 16;
    o.transpose_max = 16;
    o.wave_queue_rays = 1u << 25;
    o.diag = 0;
    o.ring_pass_bytes = 384ull << 20;
    return o;
}

int check_options(const rt_options &o)
{
    auto bad = [](const char *field) { return fail(RT_ERR_INVALID, std::string("rt_options: bad ") + field); };
    if (o.size != sizeof(rt_options)) return bad("size (set it to sizeof(rt_options))");
    if (o.render_streams > kMaxBufs) return bad("render_streams (0..8)");
    if (o.workspaces_per_stream < 1 || o.workspaces_per_stream > kMaxWs / kMaxBufs) return bad("workspaces_per_stream (1..2)");
    if (o.deep_split > 1024) return bad("deep_split (0..1024)");
    if (o.max_pass_bytes < 12 || o.max_pass_bytes > kMaxSlotsBytes) return bad("max_pass_bytes (12 B..2 GiB)");
    if (o.ring_pass_bytes && (o.ring_pass_bytes < 12 || o.ring_pass_bytes > kMaxSlotsBytes))
        return bad("ring_pass_bytes (0 or 12 B..2 GiB)");
    if (o.cluster_size < 4 || o.cluster_size > 64 || o.cluster_size % 4) return bad("cluster_size (4..64, multiple of 4)");
    if (o.transpose_max > 16) return bad("transpose_max (0..16)");
    if (o.wave_queue_rays < 64) return bad("wave_queue_rays (>= 64)");
    if (o.diag & ~((RT_DIAG_SKY_SERIAL << 1) - 1u)) return bad("diag (unknown bit)");
    if ((o.diag & RT_DIAG_SHADE_LDS) && (o.diag & RT_DIAG_SHADE_GLOBAL)) return bad("diag (shade_lds with shade_global)");
    return RT_OK;
}

int parse_options(const char *text, rt_options &o)
{
    static const struct { const char *name; uint32_t bit; } kDiag[] = {
        {"ieee_roots", RT_DIAG_IEEE_ROOTS}, {"no_shortcut", RT_DIAG_NO_SHORTCUT},
        {"no_neighbours", RT_DIAG_NO_NEIGHBOURS}, {"no_root_box", RT_DIAG_NO_ROOT_BOX},
        {"shade_lds", RT_DIAG_SHADE_LDS}, {"shade_global", RT_DIAG_SHADE_GLOBAL}, {"stats", RT_DIAG_STATS},
        {"stats_deep_only", RT_DIAG_STATS_DEEP_ONLY}, {"verbose", RT_DIAG_VERBOSE},
        {"standin_transport", RT_DIAG_STANDIN_TRANSPORT}, {"unbounded_nb", RT_DIAG_UNBOUNDED_NB},
        {"no_pairs", RT_DIAG_NO_PAIRS}, {"pairs", RT_DIAG_PAIRS}, {"in_flight", RT_DIAG_IN_FLIGHT},
        {"natural_order", RT_DIAG_NATURAL_ORDER}, {"no_sky", RT_DIAG_NO_SKY}, {"lone_unsplit", RT_DIAG_LONE_UNSPLIT},
        {"sky_serial", RT_DIAG_SKY_SERIAL}};
    rt_options n = o;
    std::string all(text ? text : "");
    for (char &c : all)
        if (c == ';' || c == ' ' || c == '\t' || c == '\n') c = ',';
    size_t pos = 0;
    while (pos <= all.size()) {
        const size_t end = std::min(all.find(',', pos), all.size());
        const std::string item = all.substr(pos, end - pos);
        pos = end + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos || eq == 0 || eq + 1 == item.size())
            return fail(RT_ERR_INVALID, "rt_options_parse: expected key=value, got '" + item + "'");
        const std::string key = item.substr(0, eq), val = item.substr(eq + 1);
        char *stop = nullptr;
        errno = 0;
        const unsigned long long v = std::strtoull(val.c_str(), &stop, 0);
        if (errno || !stop || *stop || val[0] == '-')
            return fail(RT_ERR_INVALID, "rt_options_parse: bad value for " + key + ": '" + val + "'");
        auto u32 = [&](uint32_t &f) {
            if (v > 0xffffffffull) return false;
            f = static_cast<uint32_t>(v);
            return true;
        };
        bool ok = true, known = true;
        if (key == "render_streams") ok = u32(n.render_streams);
        else if (key == "workspaces_per_stream") ok = u32(n.workspaces_per_stream);
        else if (key == "deep_split") ok = u32(n.deep_split);
        else if (key == "max_pass_bytes") n.max_pass_bytes = v;
        else if (key == "max_workspace_bytes") n.max_workspace_bytes = v;
        else if (key == "ring_pass_bytes") n.ring_pass_bytes = v;
        else if (key == "deep_min_items") n.deep_min_items = v;
        else if (key == "cluster_size") ok = u32(n.cluster_size);
        else if (key == "transpose_max") ok = u32(n.transpose_max);
        else if (key == "wave_queue_rays") ok = u32(n.wave_queue_rays);
        else if (key == "diag") ok = u32(n.diag);
        else {
            known = false;
            for (const auto &d : kDiag)
                if (key == d.name) {
                    known = true;
                    ok = v <= 1;
                    n.diag = v ? (n.diag | d.bit) : (n.diag & ~d.bit);
                }
        }
        if (!known) return fail(RT_ERR_INVALID, "rt_options_parse: unknown key '" + key + "'");
        if (!ok) return fail(RT_ERR_INVALID, "rt_options_parse: value out of range for " + key);
    }
    if (int rc = check_options(n); rc) return rc;
    o = n;
    return RT_OK;
}

// the process default for scenes created without explicit options: the library defaults with
// RT_OPTIONS applied (once; a malformed RT_OPTIONS makes every such creation fail loudly)
namespace {
std::mutex g_opt_mu;
bool g_opt_init = false;
rt_options g_opt;
std::string g_opt_env_error;
} // namespace
int default_options(rt_options &out)
{
    std::lock_guard<std::mutex> g(g_opt_mu);
    if (!g_opt_init) {
        g_opt = library_defaults();
        if (const char *e = std::getenv("RT_OPTIONS"); e && *e) {
            rt_options o = g_opt;
            if (parse_options(e, o) == RT_OK) g_opt = o;
            else g_opt_env_error = "RT_OPTIONS: " + g_error;
        }
        g_opt_init = true;
    }
    if (!g_opt_env_error.empty()) return fail(RT_ERR_INVALID, g_opt_env_error);
    out = g_opt;
    return RT_OK;
}

} // namespace rthost

extern "C" {

int rt_version(void) { return RT_API_VERSION; }

const char *rt_last_error(void) { return g_error.c_str(); }

int rt_options_default(rt_options *out)
{
    if (!out) return fail(RT_ERR_INVALID, "rt_options_default: null");
    *out = library_defaults();
    return RT_OK;
}

int rt_options_parse(const char *text, rt_options *inout)
{
    if (!text || !inout) return fail(RT_ERR_INVALID, "rt_options_parse: null argument");
    if (int rc = check_options(*inout); rc) return rc;
    return parse_options(text, *inout);
}

int rt_set_default_options(const rt_options *options)
{
    const rt_options o = options ? *options : library_defaults();
    if (int rc = check_options(o); rc) return rc;
    std::lock_guard<std::mutex> g(g_opt_mu);
    g_opt = o;
    g_opt_init = true;
    g_opt_env_error.clear();  // an explicit default replaces a malformed RT_OPTIONS
    return RT_OK;
}

int rt_get_default_options(rt_options *out)
{
    if (!out) return fail(RT_ERR_INVALID, "rt_get_default_options: null");
    return default_options(*out);
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
    // src/main.cxx:131-177 (namespace typo fixed). Draw order: type, center.x, center.z, then
    // the material's draws; a type-3 sphere pushes no material, so it shares the index of the
    // next pushed one and trailing ones are resolved by default materials (lambert, albedo 1).
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

} // namespace

namespace rthost {

// ---- scene blob: always-tested list + spatial clusters -------------------

constexpr float kPadRel = 1e-3f;      // must match RT_PAD_REL in rt_kernel.hip

// recursive median splits into clusters of at most cluster_max spheres (rt_options.cluster_size,
// 16 by default: two blocks of 8; 8 / 12 / 20 / 24 measured slower, profiles/r03/ab/knobs2_s3.txt)
void split_clusters(const rt_sphere *s, std::vector<uint32_t> ids, std::vector<std::vector<uint32_t>> &out,
                    uint32_t kClusterMax)
{
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
    split_clusters(s, std::move(left), out, kClusterMax);
    split_clusters(s, std::move(right), out, kClusterMax);
}

#ifndef RT_SUPER_FULL
#define RT_SUPER_FULL 0  // A/B build switch: every level-2 box's clusters walked, empty ones too
#endif
constexpr bool kSuperCount = RT_SUPER_FULL != 0;
blob_t build_blob(const rt_sphere *s, uint32_t n, bool clustered, uint32_t cluster_max)
{
    // three classes by |r| against the median: huge (> 64x, e.g. the ground) are tested on
    // every segment; big (> 4x) and small are clustered separately so that one big sphere
    // does not inflate the boxes of the small ones
    std::vector<uint32_t> always, big, small;
    if (clustered && n >= 2 * cluster_max) {
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
    // clusters: the big ones, padded to a multiple of kSuperClusters (an empty slot never
    // passes), then the small ones; each group of kSuperClusters consecutive clusters gets a
    // level-2 box
    std::vector<std::vector<uint32_t>> clusters;
    if (!big.empty()) split_clusters(s, big, clusters, cluster_max);
    while (clusters.size() % rt::kSuperClusters) clusters.emplace_back();
    if (!small.empty()) split_clusters(s, small, clusters, cluster_max);
    // clusters stay in the DFS order of the median-split tree: 8 consecutive clusters are a
    // depth-3 subtree, spatially tight, and become one level-2 box

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
    // pad to a multiple of kSuperClusters clusters (grouped box tests) with boxes no ray enters:
    // negative extents make t_in > t_out whatever the ray
    while (b.n_clusters % rt::kSuperClusters) {
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
    // level 2: one box over every kSuperClusters consecutive clusters (padding clusters contribute nothing)
    b.supers_offset = static_cast<uint32_t>(b.data.size() / 4);
    for (uint32_t g = 0; g < b.n_clusters; g += rt::kSuperClusters) {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t c = g; c < std::min(g + rt::kSuperClusters, b.n_clusters_real); ++c)
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
        // the clusters the walk tests under this box: up to its last non-empty one, in pairs (the
        // big spheres' group is padded to kSuperClusters with empty clusters no ray enters)
        uint32_t cn = kSuperCount ? rt::kSuperClusters : 0u;
        if (!kSuperCount) {
            for (uint32_t c = g; c < std::min(g + rt::kSuperClusters, b.n_clusters_real); ++c)
                if (!clusters[c].empty()) cn = c - g + 1u;
            cn = (cn + 1u) & ~1u;
        }
        uint32_t packed = g | (cn << 16);
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
std::vector<uint32_t> shortcut_words(const rt_sphere *s, uint32_t n, const rt_material *m, const blob_t &b,
                                     bool nb_off)
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

// ---- tile classes --------------------------------------------------------
scene_geom scene_geometry(const rt_sphere *s, const blob_t &b)
{
    scene_geom g;
    for (uint32_t i : b.always) g.always.push_back(s[i]);
    g.clus_pad = b.clus_pad;
    // cluster records {C, E, pad, start | count << 16} at clus_offset, 8 floats each
    for (uint32_t c = 0; c < b.n_clusters; ++c) {
        const float *r = b.data.data() + 4u * b.clus_offset + 8u * c;
        uint32_t packed;
        std::memcpy(&packed, r + 7, 4);
        if ((packed >> 16) == 0u || !(r[3] >= 0.f)) continue;  // empty or padding cluster
        g.boxes.insert(g.boxes.end(), r, r + 6);
    }
    if (b.n_clusters) {
        // the level-3 box follows the n_supers level-2 boxes
        const float *r = b.data.data() + 4u * b.supers_offset + 8u * b.n_supers;
        if (r[3] >= 0.f) {
            std::copy(r, r + 6, g.root);
            g.has_root = true;
        }
    }
    return g;
}

namespace {
// closed intervals in double: every operation's result contains every value its operands can take
struct iv {
    double lo, hi;
};
iv operator+(iv a, iv b) { return {a.lo + b.lo, a.hi + b.hi}; }
iv operator-(iv a, iv b) { return {a.lo - b.hi, a.hi - b.lo}; }
iv operator-(iv a, double c) { return {a.lo - c, a.hi - c}; }
iv operator*(iv a, iv b)
{
    const double p[4] = {a.lo * b.lo, a.lo * b.hi, a.hi * b.lo, a.hi * b.hi};
    return {std::min(std::min(p[0], p[1]), std::min(p[2], p[3])), std::max(std::max(p[0], p[1]), std::max(p[2], p[3]))};
}
iv operator*(double c, iv a) { return c >= 0 ? iv{c * a.lo, c * a.hi} : iv{c * a.hi, c * a.lo}; }
iv sq(iv a)
{
    if (a.lo >= 0) return {a.lo * a.lo, a.hi * a.hi};
    if (a.hi <= 0) return {a.hi * a.hi, a.lo * a.lo};
    return {0.0, std::max(a.lo * a.lo, a.hi * a.hi)};
}
iv grow(iv a, double e) { return {a.lo - e, a.hi + e}; }
double mag(iv a) { return std::max(std::fabs(a.lo), std::fabs(a.hi)); }

// Every ray o + t d (t >= 0) with o in the box o[], d in the box d[] misses the box [lo, hi]:
// the t for which a coordinate of some ray of the beam can lie in the slab form one interval
// per axis (o_lo + t d_lo <= hi and o_hi + t d_hi >= lo), which contains each single ray's
// slab interval; if the three have no common t >= 0, no ray of the beam meets the box.
bool beam_misses(const iv o[3], const iv d[3], const double lo[3], const double hi[3])
{
    double t0 = 0.0, t1 = INFINITY;
    for (int k = 0; k < 3; ++k) {
        const double a = hi[k] - o[k].lo;  // t d_lo <= a
        if (d[k].lo > 0) t1 = std::min(t1, a / d[k].lo);
        else if (d[k].lo < 0) t0 = std::max(t0, a / d[k].lo);
        else if (a < 0) return true;
        const double b = lo[k] - o[k].hi;  // t d_hi >= b
        if (d[k].hi > 0) t0 = std::max(t0, b / d[k].hi);
        else if (d[k].hi < 0) t1 = std::min(t1, b / d[k].hi);
        else if (b > 0) return true;
    }
    // empty with a relative margin far above the double divisions' rounding
    return t1 < 0 || t0 > t1 * (1 + 1e-9) + 1e-12;
}

// No ray of the beam gets a candidate from sphere S in the kernel's binary32 test
// (raytracer.hxx:52-92 as rt_kernel.hip test_block8 evaluates it), proven in exact arithmetic
// with margins of 1e-5 of the terms' magnitudes, where the binary32 evaluation errs by < 2^-21:
// either the discriminant b^2 - a c is negative for every ray, or every ray starts outside S
// (c > 0) moving away from it (b > 0) with b 2^-22 < kMIN a / 2, so that both roots are negative
// and the rounded far root stays below kMIN (the kernel's own shortcut for the ground, whose
// condition the float values then meet too).
bool sphere_missed(const iv o[3], const iv d[3], const rt_sphere &S)
{
    const iv oc[3] = {o[0] - static_cast<double>(S.center[0]), o[1] - static_cast<double>(S.center[1]),
                      o[2] - static_cast<double>(S.center[2])};
    const double r2 = static_cast<double>(S.radius) * S.radius;
    const iv a = sq(d[0]) + sq(d[1]) + sq(d[2]);
    const iv b = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
    const iv c = (sq(oc[0]) + sq(oc[1]) + sq(oc[2])) - r2;
    const double bm = mag(oc[0]) * mag(d[0]) + mag(oc[1]) * mag(d[1]) + mag(oc[2]) * mag(d[2]);
    const double cm = mag(oc[0]) * mag(oc[0]) + mag(oc[1]) * mag(oc[1]) + mag(oc[2]) * mag(oc[2]) + r2;
    const iv disc = sq(b) - a * c;
    if (disc.hi < -1e-5 * (bm * bm + a.hi * cm)) return true;
    return b.lo > 1e-5 * bm && c.lo > 1e-5 * cm && b.hi * 0x1p-22 < 0.5 * 0.008 * a.lo;
}
} // namespace

tile_order classify_tiles(const rt_camera &cam, uint32_t W, uint32_t H, uint32_t row_offset, uint32_t row_stride,
                          uint32_t num_rows, uint32_t tile_lw, const scene_geom &g, bool sky_only)
{
    tile_order out;
    const uint64_t n_pixels = static_cast<uint64_t>(W) * num_rows;
    if (!W || !H || n_pixels == 0 || n_pixels % 64u || tile_lw > 6u) return out;  // natural order
    const uint32_t n_blocks = static_cast<uint32_t>(n_pixels / 64u);
    const uint32_t tw = 1u << tile_lw, th = 64u >> tile_lw;
    const bool tiled = W % tw == 0u;
    const uint32_t tiles_x = tiled ? W / tw : 1u, tiled_rows = tiled ? (num_rows / th) * th : 0u;
    const uint32_t n_tiles = tiled ? tiles_x * (tiled_rows / th) : 0u;
    const uint32_t st = row_stride ? row_stride : 1u;
    std::vector<uint8_t> cls(n_blocks, 1);  // 0 lead, 1 other, 2 sky; untiled blocks stay 1
    const double lens = std::fabs(static_cast<double>(cam.lens_radius));
    auto classify_one = [&](uint32_t t) {
        const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
        const double x0 = static_cast<double>(tx) * tw, x1 = x0 + tw;  // x in [x0, x1), jitter < 1
        const double y0 = row_offset + static_cast<double>(ty) * th * st, y1 = y0 + static_cast<double>(th - 1) * st + 1;
        // uu = x/W + U/W, vv = y/H + U/H in binary32 (a few ulps around the exact values)
        const iv uu = grow({x0 / W, x1 / W}, 1e-6 * (x1 / W) + 1e-12);
        const iv vv = grow({y0 / H, y1 / H}, 1e-6 * (y1 / H) + 1e-12);
        const iv omv = iv{1.0, 1.0} - vv;
        // lens offset {uu rd.x, vv rd.y, 0}, |rd_k| <= lens (camera.hxx:52-54)
        const double ox = lens * mag(uu), oy = lens * mag(vv);
        const iv off[3] = {{-ox, ox}, {-oy, oy}, {0.0, 0.0}};
        iv o[3], d[3];
        for (int k = 0; k < 3; ++k) {
            const double org = cam.origin[k], llc = cam.lower_left_corner[k], hor = cam.horizontal[k], ver = cam.vertical[k];
            o[k] = grow(iv{org, org} + off[k], 1e-6 * (std::fabs(org) + mag(off[k])) + 1e-30);
            // camera.hxx:56: llc + hor u + ver (1 - v) - offset (- origin in the corrected mode)
            iv dk = ((iv{llc, llc} + hor * uu) + ver * omv) - off[k];
            double m = std::fabs(llc) + std::fabs(hor) * mag(uu) + std::fabs(ver) * mag(omv) + mag(off[k]);
            if (cam.mode == RT_CAMERA_CORRECTED) {
                dk = dk - org;
                m += std::fabs(org);
            }
            d[k] = grow(dk, 1e-5 * m + 1e-30);
        }
        const double o1 = mag(o[0]) + mag(o[1]) + mag(o[2]);
        // twice the kernel's per-ray pad (rt_kernel.hip closest_hit: 1e-3 |o|_1 + clus_pad)
        const double pad = 2.0 * (1e-3 * o1 + g.clus_pad) + 1e-6;
        auto misses_box = [&](const float *r) {
            double lo[3], hi[3];
            for (int k = 0; k < 3; ++k) {
                lo[k] = static_cast<double>(r[k]) - r[3 + k] - pad;
                hi[k] = static_cast<double>(r[k]) + r[3 + k] + pad;
            }
            return beam_misses(o, d, lo, hi);
        };
        bool sky = !g.has_root || misses_box(g.root);
        for (size_t i = 0; sky && i < g.always.size(); ++i) sky = sphere_missed(o, d, g.always[i]);
        if (sky) {
            cls[t] = 2;
            return;
        }
        if (sky_only) return;
        for (size_t c = 0; c + 6 <= g.boxes.size(); c += 6)
            if (!misses_box(g.boxes.data() + c)) {
                cls[t] = 0;
                break;
            }
    };
    // a frame's first render with a camera waits for it: config 3's 14 400 tiles take 1.05-1.16 ms
    // on one core of the GPU box's host, 0.55-0.80 on 8 threads (each writes its own tiles;
    // tests/sanitize host_check runs it under TSAN)
#ifndef RT_TILE_THREADS
#define RT_TILE_THREADS 8u
#endif
    const uint32_t n_threads = n_tiles >= 4096u ? std::min(RT_TILE_THREADS, std::max(1u, std::thread::hardware_concurrency())) : 1u;
    if (n_threads > 1) {
        // tile rows interleaved over the threads: sky rows are cheap, rows over the scene dear
        std::vector<std::thread> pool;
        // (each thread runs its own copy of the closure: the captured references then sit on the
        // thread's own stack, not in a cache line the other threads' locals keep writing)
        auto rows = [&](uint32_t k) {
            const auto one = classify_one;
            for (uint32_t r = k; r * tiles_x < n_tiles; r += n_threads)
                for (uint32_t t = r * tiles_x; t < (r + 1u) * tiles_x; ++t) one(t);
        };
        for (uint32_t k = 1; k < n_threads; ++k) pool.emplace_back(rows, k);
        rows(0);
        for (auto &th : pool) th.join();
    } else {
        for (uint32_t t = 0; t < n_tiles; ++t) classify_one(t);
    }
    out.perm.reserve(n_blocks);
    for (uint8_t want = 0; want < 3; ++want)
        for (uint32_t b = 0; b < n_blocks; ++b)
            if (cls[b] == want) out.perm.push_back(b);
    out.n_lead = static_cast<uint32_t>(std::count(cls.begin(), cls.end(), 0));
    out.n_sky = static_cast<uint32_t>(std::count(cls.begin(), cls.end(), 2));
    return out;
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

} // namespace rthost

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

// The dealing order a render of this scene gives the pass described by camera + params
// (DESIGN.md §4.7): the culled blob the scene would get (default options' cluster size), then
// classify_tiles over the pass's 8x8 tiles.
int rt_tile_order(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials, uint32_t n_materials,
                  const rt_camera *camera, const rt_params *params, uint32_t *perm, uint32_t cap, uint32_t *n_blocks,
                  uint32_t *n_lead, uint32_t *n_sky)
{
    if ((n_spheres && !spheres) || !materials || !camera || !params || !n_blocks || !n_lead || !n_sky || (cap && !perm))
        return fail(RT_ERR_INVALID, "rt_tile_order: null argument");
    (void)n_materials;
    rt_options opt;
    if (int rc = default_options(opt); rc) return rc;
    const blob_t b = build_blob(spheres, n_spheres, true, opt.cluster_size);
    const scene_geom g = scene_geometry(spheres, b);
    const uint32_t st = params->row_stride ? params->row_stride : 1u;
    const uint32_t rows = params->num_rows ? params->num_rows
                          : params->row_offset >= params->height ? 0u
                                                                 : (params->height - params->row_offset + st - 1u) / st;
    const tile_order t = classify_tiles(*camera, params->width, params->height, params->row_offset, st, rows, 3u, g);
    *n_blocks = static_cast<uint32_t>(t.perm.size());
    *n_lead = t.n_lead;
    *n_sky = t.n_sky;
    if (t.perm.size() > cap) return cap ? fail(RT_ERR_CAPACITY, "rt_tile_order: perm buffer too small") : RT_OK;
    std::copy(t.perm.begin(), t.perm.end(), perm);
    return RT_OK;
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
