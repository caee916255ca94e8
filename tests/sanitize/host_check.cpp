// TEST INFRASTRUCTURE ONLY (tests/test_sanitize_cpu.py): drives the host-only half of the
// library (raytracinginoneweekend_amd/csrc/rt_host_build.cpp, compiled from the same source
// with -fsanitize=address,undefined or -fsanitize=thread by tests/sanitize/Makefile) and the CPU
// restatement (oracle/rt_oracle.cpp) through their real inputs, and checks the results against
// the reference's fixtures in tests/golden. Any sanitizer report fails the run (halt on error).
//
//   host_check host <golden dir>        scene generators vs the reference's scene dumps, camera
//                                       vs the restatement, cluster/neighbour-list builder on the
//                                       huge scene and adversarial scenes, exact-division checks,
//                                       options parser (fixed and random strings), PPM writer
//   host_check render <scene.bin> <golden.f32> W H spp depth seed row0 stride rows mode threads
//                                       the restatement's render vs a golden frame, bit for bit
//   host_check threads <scene.bin>      (TSan) the restatement on 1 and 4 threads, the exact-division
//                                       cache and the options defaults from several threads
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../raytracinginoneweekend_amd/csrc/rt_host_build.h"

extern "C" {
int oracle_render_f32(const rt_sphere *, uint32_t, const rt_material *, uint32_t, const rt_camera *, const rt_params *,
                      int rng_mode, int threads, float *out, uint64_t *segments_out);
int oracle_camera_default(uint32_t width, uint32_t height, uint32_t mode, rt_camera *out);
}

namespace {

int g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                         \
        }                                                                     \
    } while (0)

std::vector<char> read_file(const std::string &p)
{
    std::ifstream f(p, std::ios::binary);
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

// RTSC v1 scene file (raytracinginoneweekend_amd/_abi.py save_scene_file)
bool load_scene(const std::string &p, std::vector<rt_sphere> &s, std::vector<rt_material> &m)
{
    const std::vector<char> b = read_file(p);
    if (b.size() < 16) return false;
    uint32_t h[4];
    std::memcpy(h, b.data(), 16);
    if (h[0] != 0x43535452u || h[1] != 1u || b.size() != 16u + 20u * (h[2] + h[3])) return false;
    s.resize(h[2]);
    m.resize(h[3]);
    std::memcpy(s.data(), b.data() + 16, 20u * h[2]);
    std::memcpy(m.data(), b.data() + 16 + 20u * h[2], 20u * h[3]);
    return true;
}

void check_scene_generators(const std::string &golden)
{
    std::vector<rt_sphere> gs, s(1024);
    std::vector<rt_material> gm, m(1024);
    uint32_t ns = 0, nm = 0;
    CHECK(load_scene(golden + "/scene_huge_1234.bin", gs, gm));
    CHECK(rt_scene_huge(1234, s.data(), 1024, &ns, m.data(), 1024, &nm) == RT_OK);
    CHECK(ns == gs.size() && nm == gm.size());
    CHECK(ns == gs.size() && std::memcmp(s.data(), gs.data(), ns * sizeof(rt_sphere)) == 0);
    CHECK(nm == gm.size() && std::memcmp(m.data(), gm.data(), nm * sizeof(rt_material)) == 0);
    CHECK(rt_scene_huge(1234, s.data(), 10, &ns, m.data(), 1024, &nm) == RT_ERR_CAPACITY);
    CHECK(rt_scene_huge(1234, nullptr, 0, &ns, nullptr, 0, &nm) == RT_OK && ns == gs.size());
    for (uint32_t seed : {0u, 1u, 7u, 0xffffffffu}) CHECK(rt_scene_huge(seed, s.data(), 1024, &ns, m.data(), 1024, &nm) == RT_OK);
    CHECK(load_scene(golden + "/scene_simple.bin", gs, gm));
    CHECK(rt_scene_simple(s.data(), 1024, &ns, m.data(), 1024, &nm) == RT_OK);
    CHECK(ns == gs.size() && std::memcmp(s.data(), gs.data(), ns * sizeof(rt_sphere)) == 0);
    CHECK(rt_scene_cuda(s.data(), 1024, &ns, m.data(), 1024, &nm) == RT_OK && ns == 5 && nm == 4);
}

void check_cameras()
{
    for (uint32_t W : {1u, 64u, 200u, 1280u, 3840u})
        for (uint32_t H : {1u, 36u, 100u, 720u, 2160u})
            for (uint32_t mode : {0u, 1u}) {
                rt_camera a{}, b{};
                CHECK(rt_camera_default(W, H, mode, &a) == RT_OK);
                CHECK(oracle_camera_default(W, H, mode, &b) == RT_OK);
                CHECK(std::memcmp(&a, &b, sizeof a) == 0);
            }
    rt_camera c{};
    CHECK(rt_camera_default(0, 10, 0, &c) == RT_ERR_INVALID);
    CHECK(rt_camera_cuda(64, 36, &c) == RT_OK);
    const float p[3] = {1, 2, 3};
    CHECK(rt_camera_init(p, p, p, 1.f, 90.f, 0.f, 1.f, 2u, &c) == RT_ERR_INVALID);
    CHECK(rt_camera_init(nullptr, p, p, 1.f, 90.f, 0.f, 1.f, 0u, &c) == RT_ERR_INVALID);
}

// every sphere appears exactly once: in the always-tested list or in one cluster's members
void check_blob(const std::vector<rt_sphere> &s, const std::vector<rt_material> &m, bool clustered, uint32_t csize)
{
    const uint32_t n = static_cast<uint32_t>(s.size());
    const rthost::blob_t b = rthost::build_blob(s.data(), n, clustered, csize);
    CHECK(b.n_geo % 4 == 0 && b.data.size() % 4 == 0);
    CHECK(b.clus_offset * 4u <= b.data.size() && b.supers_offset * 4u <= b.data.size());
    std::vector<int> seen(n, 0);
    for (uint32_t g = 0; g < b.n_geo; ++g) {
        uint32_t id;
        std::memcpy(&id, &b.data[4u * b.n_geo + g], 4);
        if (id != 0xffffffffu) {
            CHECK(id < n);
            if (id < n) ++seen[id];
        }
    }
    for (uint32_t i = 0; i < n; ++i) CHECK(seen[i] == 1);
    // cluster records: members inside the geo list, at most the cluster size
    for (uint32_t c = 0; c < b.n_clusters; ++c) {
        uint32_t packed;
        std::memcpy(&packed, &b.data[4u * (b.clus_offset + 2u * c) + 7u], 4);
        const uint32_t start = packed & 0xffffu, cnt = packed >> 16;
        CHECK(cnt <= ((csize + 3u) & ~3u) && start + cnt <= b.n_geo);
    }
    const std::vector<uint32_t> w = rthost::shortcut_words(s.data(), n, m.data(), b, false);
    const std::vector<uint32_t> w0 = rthost::shortcut_words(s.data(), n, m.data(), b, true);
    CHECK(w.size() == n && w0.size() == n);
    for (uint32_t i = 0; i < n; ++i) {
        if (!(w[i] & rt::kShortcut)) continue;
        CHECK(m[s[i].material].kind == RT_DIELECTRIC);
        const uint32_t n0 = w[i] & 0x7fffu, n1 = (w[i] >> 15) & 0x7fffu;
        CHECK(n0 <= b.n_geo && n1 <= b.n_geo);
        CHECK(!w0[i] || (w0[i] == rt::kShortcut && !n0));  // isolated only without neighbours
    }
}

void check_builders(const std::string &golden)
{
    std::vector<rt_sphere> s;
    std::vector<rt_material> m;
    CHECK(load_scene(golden + "/scene_huge_1234.bin", s, m));
    for (uint32_t cs = 4; cs <= 64; cs += 4) check_blob(s, m, true, cs);
    check_blob(s, m, false, 16);
    {   // the huge scene's walk shortcut (155 of its 157 glass balls)
        const rthost::blob_t b = rthost::build_blob(s.data(), static_cast<uint32_t>(s.size()), true, 16);
        const std::vector<uint32_t> w = rthost::shortcut_words(s.data(), static_cast<uint32_t>(s.size()), m.data(), b, false);
        uint32_t k = 0;
        for (uint32_t x : w) k += (x & rt::kShortcut) ? 1u : 0u;
        CHECK(k >= 150 && k <= 157);
    }
    // adversarial scenes: duplicates, zero / negative / huge radii, non-finite and far centres,
    // touching glass balls, fewer spheres than a cluster
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(-20.f, 20.f);
    for (uint32_t n : {0u, 1u, 5u, 31u, 32u, 33u, 300u, 2000u}) {
        std::vector<rt_sphere> t(n);
        std::vector<rt_material> mm = {{RT_LAMBERT, {.5f, .5f, .5f}, 0.f}, {RT_DIELECTRIC, {1, 1, 1}, 1.5f},
                                       {RT_METAL, {.7f, .6f, .5f}, .2f}};
        for (uint32_t i = 0; i < n; ++i) {
            t[i] = {{U(rng), std::fabs(U(rng)) * .05f, U(rng)}, .2f, i % 3u};
            if (i % 17 == 3 && i) t[i] = t[i - 1];                       // duplicate
            if (i % 29 == 5) t[i].radius = -.15f;                       // bubble
            if (i % 41 == 7) t[i].radius = 0.f;
            if (i % 53 == 11) t[i].center[0] = 7e5f;                    // far from the origin
            if (i % 97 == 13) t[i].center[1] = INFINITY;                // non-finite
            if (i % 89 == 17) t[i].radius = 3000.f;                     // huge (always tested)
        }
        check_blob(t, mm, true, 16);
        check_blob(t, mm, true, 4);
        check_blob(t, mm, false, 16);
    }
}

// tile classes: the frame-sized classification runs on several threads (each
// writes its own tiles; TSAN checks that), a row share's on one; the frame's is a permutation,
// the same on every run, with the classes' counts in range
void check_tiles(const std::string &golden)
{
    std::vector<rt_sphere> s;
    std::vector<rt_material> m;
    CHECK(load_scene(golden + "/scene_huge_1234.bin", s, m));
    const rthost::blob_t b = rthost::build_blob(s.data(), static_cast<uint32_t>(s.size()), true, 16);
    const rthost::scene_geom g = rthost::scene_geometry(s.data(), b);
    rt_camera cam{};
    CHECK(rt_camera_default(1280, 720, RT_CAMERA_REFERENCE, &cam) == RT_OK);
    const rthost::tile_order a = rthost::classify_tiles(cam, 1280, 720, 0, 1, 720, 3u, g);
    const rthost::tile_order a2 = rthost::classify_tiles(cam, 1280, 720, 0, 1, 720, 3u, g);
    CHECK(a.perm.size() == 14400u && a.perm == a2.perm && a.n_lead == a2.n_lead && a.n_sky == a2.n_sky);
    std::vector<uint32_t> sorted = a.perm;
    std::sort(sorted.begin(), sorted.end());
    for (uint32_t i = 0; i < sorted.size(); ++i) CHECK(sorted[i] == i);
    CHECK(a.n_lead >= 161u && a.n_sky >= 10000u && a.n_lead + a.n_sky <= 14400u);
    // rows 8 j (share 0 of 8; 90 rows): 11 tile rows of 160 tiles (8 x 8 tiles over the packed rows)
    const rthost::tile_order sh = rthost::classify_tiles(cam, 1280, 720, 0, 8, 90, 3u, g);
    CHECK(sh.perm.size() == 1800u);  // 1280 x 90 / 64 blocks
    CHECK(sh.n_sky > 0u && sh.n_sky < 1800u);
}

void check_divisions()
{
    std::mt19937 rng(9);
    for (uint32_t d : {1u, 2u, 3u, 7u, 8u, 100u, 720u, 1280u, 2160u, 3840u, 65535u, 921600u, 0x7fffffffu, 0xffffffffu}) {
        const rt::UDiv u = rthost::make_udiv(d);
        for (int k = 0; k < 20000; ++k) {
            const uint32_t n = k < 10 ? 0xffffffffu - static_cast<uint32_t>(k) : rng();
            const uint32_t t = static_cast<uint32_t>((static_cast<uint64_t>(n) * u.m) >> 32);
            const uint32_t q = (t + ((n - t) >> u.s1)) >> u.s2;
            CHECK(q == n / d);
            if (q != n / d) break;
        }
    }
    for (float b : {1.f, 200.f, 100.f, 720.f, 1280.f}) CHECK(rthost::exact_by_reciprocal(b));
    CHECK(!rthost::exact_by_reciprocal(0.f) && !rthost::exact_by_reciprocal(-3.f) && !rthost::exact_by_reciprocal(NAN));
}

void check_options()
{
    rt_options o;
    CHECK(rt_options_default(&o) == RT_OK);
    CHECK(rt_options_parse("render_streams=3,max_workspace_bytes=4294967296, stats=1", &o) == RT_OK);
    CHECK(o.render_streams == 3 && o.max_workspace_bytes == (1ull << 32) && (o.diag & RT_DIAG_STATS));
    const char *bad[] = {"x", "=", "render_streams=", "=3", "render_streams=99", "cluster_size=5", "diag=999999",
                         "max_pass_bytes=18446744073709551615", "deep_split=-1", "verbose=2", ",,,render_streams=1x"};
    for (const char *b : bad) {
        rt_options t = o;
        CHECK(rt_options_parse(b, &t) == RT_ERR_INVALID);
        CHECK(std::memcmp(&t, &o, sizeof t) == 0);
        CHECK(std::strlen(rt_last_error()) > 0);
    }
    std::mt19937 rng(3);
    const char alphabet[] = "render_streams=0123456789,x;= \t_dplitagqkmbsvwe";
    for (int k = 0; k < 20000; ++k) {  // random text: never crashes, never leaves a bad record
        std::string t(rng() % 48, ' ');
        for (char &c : t) c = alphabet[rng() % (sizeof alphabet - 1)];
        rt_options r;
        rt_options_default(&r);
        if (rt_options_parse(t.c_str(), &r) == RT_OK) CHECK(rthost::check_options(r) == RT_OK);
    }
    CHECK(rt_set_default_options(&o) == RT_OK);
    rt_options d{};
    CHECK(rt_get_default_options(&d) == RT_OK && std::memcmp(&d, &o, sizeof d) == 0);
    CHECK(rt_set_default_options(nullptr) == RT_OK);
    o.size = 3;
    CHECK(rt_set_default_options(&o) == RT_ERR_INVALID);
}

void check_ppm(const std::string &golden)
{
    const std::vector<char> ref = read_file(golden + "/c1_simple_200x100_s1.ppm");
    const std::vector<char> u8 = read_file(golden + "/c1_simple_200x100_s1.u8");
    CHECK(u8.size() == 200u * 100u * 3u);
    const std::string path = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") + "/host_check_" +
                             std::to_string(static_cast<long>(::getpid())) + ".ppm";
    CHECK(rt_write_ppm(path.c_str(), reinterpret_cast<const uint8_t *>(u8.data()), 200, 100) == RT_OK);
    const std::vector<char> mine = read_file(path);
    std::remove(path.c_str());
    const std::string hdr = "P6\n200 100\n255\n";
    CHECK(mine.size() == ref.size() && std::memcmp(mine.data(), hdr.data(), hdr.size()) == 0);
    CHECK(rt_write_ppm("/nonexistent-dir/x.ppm", reinterpret_cast<const uint8_t *>(u8.data()), 200, 100) == RT_ERR_IO);
    CHECK(rt_write_ppm(path.c_str(), nullptr, 4, 4) == RT_ERR_INVALID);
}

int render(int argc, char **argv)
{
    if (argc != 14) return 2;
    std::vector<rt_sphere> s;
    std::vector<rt_material> m;
    CHECK(load_scene(argv[2], s, m));
    const std::vector<char> want = read_file(argv[3]);
    rt_params p{};
    p.width = std::stoul(argv[4]);
    p.height = std::stoul(argv[5]);
    p.spp = std::stoul(argv[6]);
    p.max_depth = std::stoul(argv[7]);
    p.seed = std::stoull(argv[8]);
    p.row_offset = std::stoul(argv[9]);
    p.row_stride = std::stoul(argv[10]);
    p.num_rows = std::stoul(argv[11]);
    const uint32_t mode = std::stoul(argv[12]);
    const int threads = std::stoi(argv[13]);
    rt_camera cam{};
    CHECK(rt_camera_default(p.width, p.height, mode, &cam) == RT_OK);
    const uint32_t rows = p.num_rows ? p.num_rows : p.height;
    std::vector<float> out(static_cast<size_t>(rows) * p.width * 3);
    uint64_t seg = 0;
    CHECK(oracle_render_f32(s.data(), static_cast<uint32_t>(s.size()), m.data(), static_cast<uint32_t>(m.size()), &cam, &p, 0,
                            threads, out.data(), &seg) == RT_OK);
    CHECK(want.size() == out.size() * 4 && std::memcmp(want.data(), out.data(), want.size()) == 0);
    CHECK(seg >= static_cast<uint64_t>(rows) * p.width * p.spp || p.max_depth == 0);
    return g_fail ? 1 : 0;
}

int threads(const std::string &scene)
{
    std::vector<rt_sphere> s;
    std::vector<rt_material> m;
    CHECK(load_scene(scene, s, m));
    rt_camera cam{};
    CHECK(rt_camera_default(64, 36, 0, &cam) == RT_OK);
    rt_params p{64, 36, 4, 64, 1234, 0, 1, 0, 0};
    std::vector<float> a(64 * 36 * 3), b(a.size());
    uint64_t sa = 0, sb = 0;
    CHECK(oracle_render_f32(s.data(), static_cast<uint32_t>(s.size()), m.data(), static_cast<uint32_t>(m.size()), &cam, &p, 0, 1,
                            a.data(), &sa) == RT_OK);
    CHECK(oracle_render_f32(s.data(), static_cast<uint32_t>(s.size()), m.data(), static_cast<uint32_t>(m.size()), &cam, &p, 0, 4,
                            b.data(), &sb) == RT_OK);
    CHECK(std::memcmp(a.data(), b.data(), a.size() * 4) == 0 && sa == sb);
    // the library's shared host state from several threads: the exact-division cache, the
    // process-default options (RT_OPTIONS parsed once), thread-local error messages
    std::vector<std::thread> pool;
    std::vector<int> ok(8, 0);
    for (int t = 0; t < 8; ++t)
        pool.emplace_back([&, t] {
            bool good = rthost::exact_by_reciprocal(static_cast<float>(100 + t % 3));
            rt_options o;
            good = good && rt_get_default_options(&o) == RT_OK;
            good = good && rt_options_parse("render_streams=99", &o) == RT_ERR_INVALID && std::strlen(rt_last_error()) > 0;
            ok[t] = good ? 1 : 0;
        });
    for (auto &t : pool) t.join();
    for (int v : ok) CHECK(v == 1);
    return g_fail ? 1 : 0;
}

} // namespace

int main(int argc, char **argv)
{
    if (argc >= 3 && std::string(argv[1]) == "host") {
        const std::string golden = argv[2];
        check_scene_generators(golden);
        check_cameras();
        check_builders(golden);
        check_tiles(golden);
        check_divisions();
        check_options();
        check_ppm(golden);
        std::printf("host_check host: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
        return g_fail ? 1 : 0;
    }
    if (argc >= 2 && std::string(argv[1]) == "render") return render(argc, argv);
    if (argc >= 3 && std::string(argv[1]) == "threads") return threads(argv[2]);
    std::fprintf(stderr, "usage: host_check host <golden> | render ... | threads <scene.bin>\n");
    return 2;
}
