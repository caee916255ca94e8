// TEST INFRASTRUCTURE ONLY — never linked into, loaded by, or called from the product.
//
// Harness around the REFERENCE's own CPU render path. It #includes the reference's
// src/main.cxx (from a portability-patched scratch copy, see oracle/build_ref.sh) and
// re-drives the pixel loop of src/main.cxx:185-215, which is dead code in the shipped
// main() (it returns at src/main.cxx:118). Every function on the hot path — app::color,
// app::background_color, app::gamma_correction, app::normalize_rgb_to_8bit,
// raytracer::hit_world/intersect/apply_material/random_in_unit_sphere/
// schlick_reflection_probability, raytracer::camera — is the reference's code, compiled
// as-is. The harness only supplies: parameters (size, spp, depth, seeds), deterministic
// seeding, a per-sample RNG engine (RT_REF_ENGINE_PCG build), the huge-scene generator
// (src/main.cxx:131-177 does not compile as shipped), and I/O.
//
// Build: oracle/build_ref.sh -> oracle/_ref/ref_harness_{mt,pcg}. Used only by
// tests/golden/make_golden.py (fixture generation) and bench.py's cpu_baseline leg.

#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <execution>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <numeric>
#include <optional>
#include <random>
#include <string>
#include <string_view>
#include <thread>
#include <tuple>
#include <variant>
#include <vector>

// The huge-scene generator uses the genuine engine whatever build this is.
using true_mt19937 = std::mt19937;

#ifdef RT_REF_ENGINE_PCG
// Per-sample PCG32 (O'Neill, pcg32_srandom_r / pcg32_random_r, XSH-RR 64/32) standing in
// for std::mt19937 in raytracer::data and raytracer::camera. Same URBG surface as
// mt19937 (32-bit output, min 0, max 2^32-1), so libstdc++'s generate_canonical consumes
// exactly one draw per uniform_real_distribution<float> call, as with mt19937.
struct rt_oracle_pcg32 {
    using result_type = std::uint32_t;
    static constexpr result_type min() { return 0u; }
    static constexpr result_type max() { return 0xffffffffu; }
    std::uint64_t state{0}, inc{1};
    rt_oracle_pcg32() = default;
    explicit rt_oracle_pcg32(std::uint64_t s) { seed(s, 0); }
    void seed(std::uint64_t initstate, std::uint64_t initseq)
    {
        state = 0u;
        inc = (initseq << 1u) | 1u;
        (*this)();
        state += initstate;
        (*this)();
    }
    result_type operator()()
    {
        std::uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        std::uint32_t xorshifted = static_cast<std::uint32_t>(((old >> 18u) ^ old) >> 27u);
        std::uint32_t rot = static_cast<std::uint32_t>(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((0u - rot) & 31u));
    }
};
namespace std { using rt_oracle_pcg32_engine = ::rt_oracle_pcg32; }
#define mt19937 rt_oracle_pcg32_engine
#endif

#define private public
#define main static reference_main
#include "main.cxx"
#undef main
#undef private

namespace harness {

struct sphere_rec { float c[3]; float r; std::uint32_t mat; };
struct material_rec { std::uint32_t kind; float albedo[3]; float param; };
static_assert(sizeof(sphere_rec) == 20 && sizeof(material_rec) == 20);

// ---- scenes -------------------------------------------------------------------------
// src/main.cxx:120-129
void scene_simple(raytracer::data &d)
{
    d.materials.push_back(material::lambert{math::vec3{.1, .2, .5}});
    d.materials.push_back(material::metal{math::vec3{.8, .6, .2}, 0});
    d.materials.push_back(material::dielectric{math::vec3{1}, 1.5f});
    d.materials.push_back(material::lambert{math::vec3{.64, .8, .0}});
    d.spheres.emplace_back(math::vec3{0, 1, 0}, 1.f, 0);
    d.spheres.emplace_back(math::vec3{0, -1000.125f, 0}, 1000.f, 3);
    d.spheres.emplace_back(math::vec3{+2, 1, 0}, 1.f, 1);
    d.spheres.emplace_back(math::vec3{-2, 1, 0}, 1.f, 2);
    d.spheres.emplace_back(math::vec3{-2, 1, 0}, -.99f, 2);
}

// src/main.cxx:131-177 with `raytracer::{lambert,metal,dielectric}` -> `material::...`
// (the shipped block references types that do not exist). Draw order is the reference's:
// braced initialisers evaluate left to right. Type 3 pushes no material, exactly as
// shipped; indices left dangling past the end are resolved by appending default
// material::types{} (lambert, albedo 1) — the only deterministic reading of that UB.
void scene_huge(raytracer::data &d, std::uint32_t seed)
{
    scene_simple(d);
    true_mt19937 generator{seed};
    auto rd_int = std::uniform_int_distribution{0, 3};
    auto rd_real = std::uniform_real_distribution{0.f, 1.f};
    for (auto a = -11; a < 11; ++a) {
        for (auto b = -11; b < 11; ++b) {
            auto material_type_index = rd_int(generator);
            math::vec3 center{.9f * rd_real(generator) + a, .2f, .9f * rd_real(generator) + b};
            if (math::distance(center, math::vec3{0, 1, 0}) < 1.f)
                continue;
            d.spheres.emplace_back(center, .2f, std::size(d.materials));
            switch (material_type_index) {
            case 0:
                d.materials.emplace_back(material::lambert{
                    math::vec3{rd_real(generator), rd_real(generator), rd_real(generator)}});
                break;
            case 1:
                d.materials.emplace_back(material::metal{
                    math::vec3{rd_real(generator), rd_real(generator), rd_real(generator)},
                    .5f * rd_real(generator)});
                break;
            case 2:
                d.materials.emplace_back(material::dielectric{
                    math::vec3{rd_real(generator), rd_real(generator), rd_real(generator)}, 1.5f});
                break;
            default:
                break;
            }
        }
    }
    std::size_t need = 0;
    for (auto &s : d.spheres) need = std::max(need, s.material_index + 1);
    while (d.materials.size() < need) d.materials.emplace_back(material::types{});
}

void scene_to_records(const raytracer::data &d, std::vector<sphere_rec> &S, std::vector<material_rec> &M)
{
    S.clear(); M.clear();
    for (auto &s : d.spheres)
        S.push_back({{s.center.x, s.center.y, s.center.z}, s.radius, static_cast<std::uint32_t>(s.material_index)});
    for (auto &m : d.materials) {
        material_rec r{};
        std::visit([&](auto &&mm) {
            using T = std::decay_t<decltype(mm)>;
            r.albedo[0] = mm.albedo.x; r.albedo[1] = mm.albedo.y; r.albedo[2] = mm.albedo.z;
            if constexpr (std::is_same_v<T, material::lambert>) { r.kind = 0; r.param = 0.f; }
            else if constexpr (std::is_same_v<T, material::metal>) { r.kind = 1; r.param = mm.roughness; }
            else { r.kind = 2; r.param = mm.refraction_index; }
        }, m);
        M.push_back(r);
    }
}

void records_to_scene(const std::vector<sphere_rec> &S, const std::vector<material_rec> &M, raytracer::data &d)
{
    d.spheres.clear(); d.materials.clear();
    for (auto &s : S) d.spheres.emplace_back(math::vec3{s.c[0], s.c[1], s.c[2]}, s.r, static_cast<std::size_t>(s.mat));
    for (auto &m : M) {
        math::vec3 alb{m.albedo[0], m.albedo[1], m.albedo[2]};
        if (m.kind == 0) d.materials.push_back(material::lambert{alb});
        else if (m.kind == 1) d.materials.push_back(material::metal{alb, m.param});
        else d.materials.push_back(material::dielectric{alb, m.param});
    }
}

// Scene file: "RTSC" u32 version=1, u32 n_spheres, u32 n_materials, records.
void save_scene(const std::string &path, const raytracer::data &d)
{
    std::vector<sphere_rec> S; std::vector<material_rec> M; scene_to_records(d, S, M);
    std::ofstream f(path, std::ios::binary);
    std::uint32_t hdr[4] = {0x43535452u, 1u, (std::uint32_t)S.size(), (std::uint32_t)M.size()};
    f.write((const char *)hdr, sizeof hdr);
    f.write((const char *)S.data(), S.size() * sizeof(sphere_rec));
    f.write((const char *)M.data(), M.size() * sizeof(material_rec));
    if (!f) throw std::runtime_error("cannot write " + path);
}

void load_scene(const std::string &path, raytracer::data &d)
{
    std::ifstream f(path, std::ios::binary);
    std::uint32_t hdr[4];
    f.read((char *)hdr, sizeof hdr);
    if (!f || hdr[0] != 0x43535452u || hdr[1] != 1u) throw std::runtime_error("bad scene file " + path);
    std::vector<sphere_rec> S(hdr[2]); std::vector<material_rec> M(hdr[3]);
    f.read((char *)S.data(), S.size() * sizeof(sphere_rec));
    f.read((char *)M.data(), M.size() * sizeof(material_rec));
    if (!f) throw std::runtime_error("short scene file " + path);
    records_to_scene(S, M, d);
}

// ---- render -------------------------------------------------------------------------
struct args_t {
    std::string scene = "simple";
    std::uint32_t scene_seed = 1234;
    std::uint32_t W = 200, H = 100, spp = 1, depth = 64;
    std::uint64_t seed = 1234;
    bool corrected = false;
    std::uint32_t row0 = 0, nrows = 0, row_step = 1;
    unsigned threads = 1;
    std::string out_f32, out_u8, out_ppm, dump_scene, kat, kat_out;
    std::uint32_t kat_n = 1024;
    bool timing = false;
};

// app::color (src/main.cxx:52-75) is called verbatim at the reference's 64 bounces; any
// other depth (config 2 asks for 50) re-drives the same loop with the bound as a
// parameter — bounces_number is a static constexpr in the reference.
math::vec3 color_depth(raytracer::data &d, math::ray ray, std::uint32_t depth)
{
    if (depth == raytracer::data::bounces_number) return app::color(d, ray);
    math::vec3 attenuation{1};
    auto scattered_ray = ray;
    math::vec3 energy_absorption{0};
    for (auto bounce = 0u; bounce < depth; ++bounce) {
        auto hit = raytracer::hit_world(d.spheres, scattered_ray);
        if (!hit) return app::background_color(.5f * scattered_ray.unit_direction().y + 1.f) * attenuation;
        auto scattered = raytracer::apply_material(d, scattered_ray, hit.value());
        if (!scattered) return math::vec3{0};
        std::tie(scattered_ray, energy_absorption) = *scattered;
        attenuation *= energy_absorption;
    }
    return math::vec3{0};
}

raytracer::camera make_camera(const args_t &a)
{
    // src/main.cxx:179-183
    return raytracer::camera{
        math::vec3{-4, 3.2, 5}, math::vec3{0, 1, 0}, math::vec3{0, 1, 0},
        static_cast<float>(a.W) / static_cast<float>(a.H), 42.f,
        0.0625f, math::distance(math::vec3{-4, 3.2, 5}, math::vec3{0, 1, 0})};
}

// Renders rows y = row0 + i*row_step, i < nrows, of the W x H frame; threads take runs of 64
// pixels of those rows from a shared counter (dynamic, so that 256 threads stay busy on a
// frame of 720 rows of uneven cost; PCG build only: the verbatim mt19937 build shares one
// stream across the frame and must run on one thread, as the reference does).
void render(const args_t &a, const std::vector<sphere_rec> &S, const std::vector<material_rec> &M,
            std::vector<float> &f32, std::vector<std::uint8_t> &u8)
{
    const std::uint32_t nrows = a.nrows;
    f32.assign((std::size_t)nrows * a.W * 3, 0.f);
    u8.assign((std::size_t)nrows * a.W * 3, 0);
    unsigned T = a.threads;
#ifndef RT_REF_ENGINE_PCG
    T = 1;
#endif
    std::atomic<std::uint64_t> next_run{0};
    auto worker = [&](unsigned tid) {
        raytracer::data raytracer_data;
        records_to_scene(S, M, raytracer_data);
        raytracer::camera camera = make_camera(a);
#ifndef RT_REF_ENGINE_PCG
        raytracer_data.generator.seed(static_cast<std::uint32_t>(a.seed));
        camera.generator.seed(static_cast<std::uint32_t>(a.seed + 1));
#endif
        std::vector<math::vec3> multisampling_texels(a.spp, math::vec3{0});
        auto random_distribution = std::uniform_real_distribution{0.f, 1.f};
        (void)tid;
        const std::uint32_t runs_per_row = (a.W + 63u) / 64u;
        for (;;) {
            const std::uint64_t run = next_run.fetch_add(1, std::memory_order_relaxed);
            if (run >= (std::uint64_t)nrows * runs_per_row) break;
            const std::uint32_t i = static_cast<std::uint32_t>(run / runs_per_row);
            const std::uint32_t x0 = static_cast<std::uint32_t>(run % runs_per_row) * 64u;
            const std::uint32_t y = a.row0 + i * a.row_step;
            auto v = static_cast<float>(y) / static_cast<float>(a.H);
            for (auto x = x0; x < std::min(a.W, x0 + 64u); ++x) {
                auto u = static_cast<float>(x) / static_cast<float>(a.W);
                std::uint32_t s = 0;
                std::generate(std::execution::par, std::begin(multisampling_texels), std::end(multisampling_texels), [&]() {
#ifdef RT_REF_ENGINE_PCG
                    const std::uint64_t key = ((std::uint64_t)y * a.W + x) * a.spp + s;
                    raytracer_data.generator.seed(key, 2u * a.seed);
                    camera.generator.seed(key, 2u * a.seed + 1u);
#endif
                    ++s;
                    auto _u = u + random_distribution(raytracer_data.generator) / static_cast<float>(a.W);
                    auto _v = v + random_distribution(raytracer_data.generator) / static_cast<float>(a.H);
                    math::ray r = camera.ray(_u, _v);
                    if (a.corrected) r.direction = r.direction - camera.origin;
                    return color_depth(raytracer_data, r, a.depth);
                });
                auto color = std::reduce(std::execution::seq, std::begin(multisampling_texels), std::end(multisampling_texels), math::vec3{0});
                color /= static_cast<float>(a.spp);
                const std::size_t o = ((std::size_t)i * a.W + x) * 3;
                f32[o + 0] = color.x; f32[o + 1] = color.y; f32[o + 2] = color.z;
                color = app::gamma_correction(color);
                auto rgb = app::normalize_rgb_to_8bit(std::move(color));
                u8[o + 0] = rgb.x; u8[o + 1] = rgb.y; u8[o + 2] = rgb.z;
            }
        }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < T; ++t) pool.emplace_back(worker, t);
    worker(0);
    for (auto &t : pool) t.join();
}

// ---- known-answer tables (PCG build) ------------------------------------------------
// Every record is a row of 32-bit words; floats are stored by bit pattern.
struct kat_writer {
    std::vector<std::uint32_t> words;
    void f(float x) { std::uint32_t w; std::memcpy(&w, &x, 4); words.push_back(w); }
    void u(std::uint32_t x) { words.push_back(x); }
    void v3(const math::vec3 &x) { f(x.x); f(x.y); f(x.z); }
    void save(const std::string &p) { std::ofstream o(p, std::ios::binary); o.write((const char *)words.data(), words.size() * 4); }
};

#ifdef RT_REF_ENGINE_PCG
// hit_world over the scene for random rays. Row: o[3] d[3] | hit mat_or_ffffffff t pos[3] normal[3]
void kat_hit(const args_t &a, raytracer::data &d, kat_writer &w)
{
    rt_oracle_pcg32 g; g.seed(a.kat_n, 99);
    auto U = std::uniform_real_distribution{-1.f, 1.f};
    for (std::uint32_t i = 0; i < a.kat_n; ++i) {
        math::vec3 o{4.f * U(g), 1.5f + 2.f * U(g), 4.f * U(g)};
        math::vec3 dir{U(g), U(g), U(g)};
        if (i % 4 == 1) { // secondary-ray shape: start on a sphere surface
            auto &s = d.spheres[i % d.spheres.size()];
            auto n = math::normalize(math::vec3{U(g), U(g), U(g)});
            o = s.center + n * s.radius;
        }
        if (i % 16 == 3) dir = dir * 1e-3f; // short, unnormalised directions
        math::ray r{o, dir};
        auto h = raytracer::hit_world(d.spheres, r);
        w.v3(o); w.v3(dir);
        if (h) { w.u((std::uint32_t)h->material_index); w.f(h->time); w.v3(h->position); w.v3(h->normal); }
        else { w.u(0xffffffffu); w.f(0.f); w.v3(math::vec3{0}); w.v3(math::vec3{0}); }
    }
}

// apply_material for random hits. Row: mat d[3] pos[3] n[3] key |
//   valid o[3] dir[3] atten[3] draws_state_lo draws_state_hi
void kat_scatter(const args_t &a, raytracer::data &d, kat_writer &w)
{
    rt_oracle_pcg32 g; g.seed(a.kat_n, 77);
    auto U = std::uniform_real_distribution{-1.f, 1.f};
    for (std::uint32_t i = 0; i < a.kat_n; ++i) {
        std::uint32_t mat = i % d.materials.size();
        math::vec3 dir{U(g), U(g), U(g)};
        math::vec3 pos{3.f * U(g), 3.f * U(g), 3.f * U(g)};
        math::vec3 n = math::normalize(math::vec3{U(g), U(g), U(g)});
        if (i % 8 == 5) n = -n; // back faces: inside a dielectric / below a metal
        if (i % 8 == 6) { // grazing: drive total internal reflection
            n = math::normalize(math::vec3{U(g), U(g), U(g)});
            dir = n * .05f + math::normalize(math::cross(n, math::vec3{.3f, .5f, .7f}));
        }
        primitives::hit h{pos, n, 1.f, mat};
        math::ray r{math::vec3{0}, dir};
        d.generator.seed(i, 5);
        auto res = raytracer::apply_material(d, r, h);
        w.u(mat); w.v3(dir); w.v3(pos); w.v3(n); w.u(i);
        if (res) { w.u(1); w.v3(res->first.origin); w.v3(res->first.direction); w.v3(res->second); }
        else { w.u(0); w.v3(math::vec3{0}); w.v3(math::vec3{0}); w.v3(math::vec3{0}); }
        w.u((std::uint32_t)d.generator.state); w.u((std::uint32_t)(d.generator.state >> 32));
    }
}

// camera::ray. Row: u v key | o[3] d[3]
void kat_camera(const args_t &a, kat_writer &w)
{
    raytracer::camera cam = make_camera(a);
    rt_oracle_pcg32 g; g.seed(a.kat_n, 55);
    auto U = std::uniform_real_distribution{0.f, 1.f};
    for (std::uint32_t i = 0; i < a.kat_n; ++i) {
        float u = U(g), v = U(g);
        cam.generator.seed(i, 3);
        auto r = cam.ray(u, v);
        w.f(u); w.f(v); w.u(i); w.v3(r.origin); w.v3(r.direction);
    }
    // the basis itself, last row: origin llc horizontal vertical lens_radius
    w.v3(cam.origin); w.v3(cam.lower_left_corner); w.v3(cam.horizontal); w.v3(cam.vertical); w.f(cam.lens_radius);
}

// background / gamma / u8 / refract / reflect / schlick.
// Row: t c[3] I[3] N[3] eta cos | bg[3] gamma[3] u8[3] refract[3] reflect[3] schlick
void kat_misc(const args_t &a, kat_writer &w)
{
    rt_oracle_pcg32 g; g.seed(a.kat_n, 33);
    auto U = std::uniform_real_distribution{0.f, 1.f};
    auto S = std::uniform_real_distribution{-1.f, 1.f};
    for (std::uint32_t i = 0; i < a.kat_n; ++i) {
        float t = .5f + U(g);
        math::vec3 c{U(g), U(g), U(g)};
        if (i % 7 == 0) c = math::vec3{1.f, 0.f, U(g) * 1e-3f};
        math::vec3 I = math::normalize(math::vec3{S(g), S(g), S(g)});
        math::vec3 N = math::normalize(math::vec3{S(g), S(g), S(g)});
        float eta = (i & 1) ? 1.5f : 1.f / 1.5f;
        float cosv = U(g);
        auto bg = app::background_color(t);
        auto gm = app::gamma_correction(c);
        auto q = app::normalize_rgb_to_8bit(gm);
        auto rf = math::refract(I, N, eta);
        auto rl = math::reflect(I, N);
        float sc = raytracer::schlick_reflection_probability(eta, cosv);
        w.f(t); w.v3(c); w.v3(I); w.v3(N); w.f(eta); w.f(cosv);
        w.v3(bg); w.v3(gm); w.u(q.x); w.u(q.y); w.u(q.z); w.v3(rf); w.v3(rl); w.f(sc);
    }
}
#endif

int run(int argc, char **argv)
{
    args_t a;
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i];
        auto nxt = [&]() -> std::string { if (i + 1 >= argc) throw std::runtime_error("missing value for " + k); return argv[++i]; };
        if (k == "--scene") a.scene = nxt();
        else if (k == "--scene-seed") a.scene_seed = std::stoul(nxt());
        else if (k == "--w") a.W = std::stoul(nxt());
        else if (k == "--h") a.H = std::stoul(nxt());
        else if (k == "--spp") a.spp = std::stoul(nxt());
        else if (k == "--depth") a.depth = std::stoul(nxt());
        else if (k == "--seed") a.seed = std::stoull(nxt());
        else if (k == "--camera") { auto m = nxt(); a.corrected = (m == "corrected"); }
        else if (k == "--row0") a.row0 = std::stoul(nxt());
        else if (k == "--rows") a.nrows = std::stoul(nxt());
        else if (k == "--row-step") a.row_step = std::stoul(nxt());
        else if (k == "--threads") a.threads = std::max(1ul, std::stoul(nxt()));
        else if (k == "--out-f32") a.out_f32 = nxt();
        else if (k == "--out-u8") a.out_u8 = nxt();
        else if (k == "--out-ppm") a.out_ppm = nxt();
        else if (k == "--dump-scene") a.dump_scene = nxt();
        else if (k == "--kat") a.kat = nxt();
        else if (k == "--kat-out") a.kat_out = nxt();
        else if (k == "--kat-n") a.kat_n = std::stoul(nxt());
        else if (k == "--time") a.timing = true;
        else throw std::runtime_error("unknown argument " + k);
    }
    raytracer::data scene;
    if (a.scene == "simple") scene_simple(scene);
    else if (a.scene == "huge") scene_huge(scene, a.scene_seed);
    else load_scene(a.scene, scene);
    if (!a.dump_scene.empty()) save_scene(a.dump_scene, scene);

    if (!a.kat.empty()) {
#ifdef RT_REF_ENGINE_PCG
        kat_writer w;
        if (a.kat == "hit") kat_hit(a, scene, w);
        else if (a.kat == "scatter") kat_scatter(a, scene, w);
        else if (a.kat == "camera") kat_camera(a, w);
        else if (a.kat == "misc") kat_misc(a, w);
        else throw std::runtime_error("unknown kat " + a.kat);
        w.save(a.kat_out);
        return 0;
#else
        throw std::runtime_error("KATs need the PCG build");
#endif
    }
    if (a.nrows == 0) a.nrows = (a.H - a.row0 + a.row_step - 1) / a.row_step;
    std::vector<sphere_rec> S; std::vector<material_rec> M; scene_to_records(scene, S, M);
    std::vector<float> f32; std::vector<std::uint8_t> u8;
    auto t0 = std::chrono::steady_clock::now();
    render(a, S, M, f32, u8);
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!a.out_f32.empty()) { std::ofstream o(a.out_f32, std::ios::binary); o.write((const char *)f32.data(), f32.size() * 4); }
    if (!a.out_u8.empty()) { std::ofstream o(a.out_u8, std::ios::binary); o.write((const char *)u8.data(), u8.size()); }
    if (!a.out_ppm.empty()) {
        // the reference's own writer, app::save_to_file (src/main.cxx:87-101)
        app::data ad;
        ad.width = a.W;
        ad.height = a.nrows;
        std::vector<math::u8vec3> tex(u8.size() / 3);
        for (size_t i = 0; i < tex.size(); ++i) {
            tex[i].x = u8[3 * i];
            tex[i].y = u8[3 * i + 1];
            tex[i].z = u8[3 * i + 2];
        }
        app::save_to_file(a.out_ppm, ad, tex);
    }
    if (a.timing) {
        double prim = (double)a.W * a.nrows * a.spp;
        std::printf("{\"seconds\": %.6f, \"primaries\": %.0f, \"mrays_per_s\": %.6f, \"threads\": %u, \"spheres\": %zu}\n",
                    sec, prim, prim / sec / 1e6, a.threads, S.size());
    }
    return 0;
}

} // namespace harness

int main(int argc, char **argv)
{
    try {
        return harness::run(argc, argv);
    } catch (std::exception &e) {
        std::fprintf(stderr, "ref_harness: %s\n", e.what());
        return 2;
    }
}
