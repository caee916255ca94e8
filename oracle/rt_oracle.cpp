// TEST INFRASTRUCTURE ONLY — the parity checker. Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library; the product (librt_mi355x.so) never
// links, loads or calls it, and has no CPU fallback.
//
// A CPU restatement of the reference's CPU render path (Alabuta/RaytracingInOneWeekend),
// written independently of both the reference's template code and our HIP kernel. Every
// arithmetic step is a separately rounded IEEE-754 binary32 operation in the reference's
// evaluation order (compiled with -ffp-contract=off; x86-64 SSE keeps denormals), so the
// result is bit-identical to the reference built by oracle/build_ref.sh. That is checked,
// not assumed: tests/test_oracle_golden.py compares this library against fixtures produced
// by the reference itself (tests/golden/make_golden.py).
//
// Citations are file:line in /root/reference.

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../include/rt_api.h"

namespace {

struct v3 { float x, y, z; };
inline v3 mk(float x, float y, float z) { return {x, y, z}; }
inline v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }        // math.hxx:79-82
inline v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }        // math.hxx:85-88
inline v3 mulv(v3 a, v3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }       // math.hxx:91-94
inline v3 muls(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }           // math.hxx:118-121
inline v3 divs(v3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }           // math.hxx:124-127
inline v3 adds(v3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }           // math.hxx:106-109
inline v3 neg(v3 a) { return {-a.x, -a.y, -a.z}; }                              // math.hxx:103
inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }     // math.hxx:278-282
inline float norm(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }          // math.hxx:209-212
inline float length(v3 a) { return std::sqrt(norm(a)); }                        // math.hxx:214-217
inline v3 normalize(v3 a)                                                       // math.hxx:219-227
{
    float l = length(a);
    if (std::fabs(l) > FLT_MIN) return divs(a, l);
    return a;
}
inline v3 cross(v3 l, v3 r)                                                     // math.hxx:284-292
{
    return {l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x};
}
inline v3 reflect(v3 I, v3 N) { return sub(I, muls(muls(N, dot(N, I)), 2.f)); } // math.hxx:294-298
inline v3 refract(v3 I, v3 N, float eta)                                        // math.hxx:300-309
{
    const float d = dot(N, I);
    const float k = 1.f - eta * eta * (1.f - d * d);
    v3 t = adds(muls(N, std::sqrt(k)), d * eta);
    return muls(sub(muls(I, eta), t), static_cast<float>(k >= 0.f));
}
inline v3 mix(v3 x, v3 y, float a) { return add(muls(x, 1.f - a), muls(y, a)); } // math.hxx:325-329

// ---- engines ----------------------------------------------------------------------
struct pcg32 {  // pcg32_srandom_r / pcg32_random_r (XSH-RR 64/32)
    std::uint64_t state = 0, inc = 1;
    void seed(std::uint64_t initstate, std::uint64_t initseq)
    {
        state = 0;
        inc = (initseq << 1u) | 1u;
        next();
        state += initstate;
        next();
    }
    std::uint32_t next()
    {
        std::uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        std::uint32_t xs = static_cast<std::uint32_t>(((old >> 18u) ^ old) >> 27u);
        std::uint32_t rot = static_cast<std::uint32_t>(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
};
struct mt { std::mt19937 g; std::uint32_t next() { return static_cast<std::uint32_t>(g()); } };

// libstdc++ generate_canonical<float, 24> over a 32-bit engine (bits/random.tcc:3348-3380):
// one draw, float(x) / 2^32, clamped below 1; uniform_real_distribution (bits/random.h:1870)
// then maps U -> U*(b-a) + a.
template <class G> inline float canonical(G &g)
{
    float r = static_cast<float>(g.next()) / 4294967296.0f;
    if (r >= 1.f) r = std::nextafter(1.f, 0.f);
    return r;
}
template <class G> inline float uniform(G &g, float a, float b) { return canonical(g) * (b - a) + a; }

template <class G> inline v3 random_in_unit_sphere(G &g)                        // raytracer.hxx:32-43
{
    v3 p;
    do {
        float x = uniform(g, -1.f, 1.f);
        float y = uniform(g, -1.f, 1.f);
        float z = uniform(g, -1.f, 1.f);
        p = mk(x, y, z);
    } while (length(p) > 1.f);
    return p;
}

inline float schlick(float ri, float c)                                        // raytracer.hxx:45-50
{
    // std::pow(float, int) promotes to double; the sum is double, returned as float.
    double r0 = std::pow(static_cast<double>((1.f - ri) / (1.f + ri)), 2.0);
    return static_cast<float>(r0 + (1.0 - r0) * std::pow(static_cast<double>(1.f - c), 5.0));
}

struct ray { v3 o, d; };
struct hit { v3 p, n; float t; std::uint32_t mat; bool ok; };

struct scene {
    const rt_sphere *s; std::uint32_t n;
    const rt_material *m; std::uint32_t nm;
};

inline bool intersect(const ray &r, const rt_sphere &sp, float tmin, float tmax, hit &h) // raytracer.hxx:52-92
{
    v3 c = mk(sp.center[0], sp.center[1], sp.center[2]);
    v3 oc = sub(r.o, c);
    float a = dot(r.d, r.d);
    float b = dot(oc, r.d);
    float cc = dot(oc, oc) - sp.radius * sp.radius;
    float disc = b * b - a * cc;
    if (disc > 0.f) {
        float t = (-b - std::sqrt(b * b - a * cc)) / a;
        if (t < tmax && t > tmin) {
            v3 p = add(r.o, muls(r.d, t));
            h = {p, divs(sub(p, c), sp.radius), t, sp.material, true};
            return true;
        }
        t = (-b + std::sqrt(b * b - a * cc)) / a;
        if (t < tmax && t > tmin) {
            v3 p = add(r.o, muls(r.d, t));
            h = {p, divs(sub(p, c), sp.radius), t, sp.material, true};
            return true;
        }
    }
    return false;
}

// raytracer.hxx:94-118: every sphere tested on (0.008, FLT_MAX); the first hit with the
// smallest time wins (stable_partition + min_element with a strict '<').
inline hit hit_world(const scene &sc, const ray &r)
{
    hit best{}; best.ok = false;
    for (std::uint32_t i = 0; i < sc.n; ++i) {
        hit h;
        if (intersect(r, sc.s[i], .008f, FLT_MAX, h) && (!best.ok || h.t < best.t)) best = h;
    }
    return best;
}

// raytracer.hxx:120-199. Returns false for "no scatter" (metal absorbed).
template <class G> inline bool apply_material(const scene &sc, G &g, const ray &r, const hit &h, ray &out, v3 &atten)
{
    const rt_material &m = sc.m[h.mat];
    v3 albedo = mk(m.albedo[0], m.albedo[1], m.albedo[2]);
    if (m.kind == RT_LAMBERT) {                                                  // :132-141
        v3 rd = random_in_unit_sphere(g);
        v3 target = add(add(h.p, h.n), rd);
        out = {h.p, sub(target, h.p)};
        atten = albedo;
        return true;
    }
    if (m.kind == RT_METAL) {                                                    // :143-156
        v3 refl = reflect(normalize(r.d), h.n);
        v3 rd = random_in_unit_sphere(g);
        out = {h.p, add(refl, muls(rd, m.param))};
        atten = albedo;
        return dot(out.d, h.n) > 0.f;
    }
    // dielectric :158-194
    v3 ud = normalize(r.d);
    v3 outward = neg(h.n);
    float ri = m.param;
    float cosv = dot(ud, h.n);
    if (cosv <= 0.f) {
        outward = muls(outward, -1.f);
        ri = 1.f / ri;
        cosv *= -1.f;
    }
    atten = albedo;
    v3 refr = refract(ud, outward, ri);
    float prob = 1.f;
    if (length(refr) > 0.f) prob = schlick(ri, cosv);
    if (canonical(g) < prob) out = {h.p, reflect(ud, h.n)};
    else out = {h.p, refr};
    return true;
}

inline v3 background(float t) { return mix(mk(1.f, 1.f, 1.f), mk(.5f, .7f, 1.f), t); } // main.cxx:47-50

struct cam {
    v3 origin, llc, hor, ver; float lens; bool corrected;
};

template <class G> inline ray camera_ray(const cam &c, G &g, float u, float v) // camera.hxx:46-57
{
    v3 rd = muls(random_in_unit_sphere(g), c.lens);
    v3 off = mk(u * rd.x, v * rd.y, 0.f);
    ray r{add(c.origin, off), sub(add(add(c.llc, muls(c.hor, u)), muls(c.ver, 1.f - v)), off)};
    if (c.corrected) r.d = sub(r.d, c.origin);
    return r;
}

// main.cxx:52-75 with the bounce bound as a parameter.
template <class G> inline v3 color(const scene &sc, G &g, ray r, std::uint32_t depth, std::uint64_t &segments)
{
    v3 atten = mk(1.f, 1.f, 1.f);
    for (std::uint32_t b = 0; b < depth; ++b) {
        ++segments;
        hit h = hit_world(sc, r);
        if (!h.ok) return mulv(background(.5f * normalize(r.d).y + 1.f), atten);
        ray nr; v3 e;
        if (!apply_material(sc, g, r, h, nr, e)) return mk(0.f, 0.f, 0.f);
        r = nr;
        atten = mulv(atten, e);
    }
    return mk(0.f, 0.f, 0.f);
}

// std::reduce(std::execution::seq, ...) -> libstdc++ transform_reduce (<numeric>:443-460):
// blocks of four as ((c0+c1)+(c2+c3)) added to the running sum, then the tail one by one.
inline v3 reduce_samples(const std::vector<v3> &c)
{
    v3 acc = mk(0.f, 0.f, 0.f);
    std::size_t i = 0, n = c.size();
    for (; n - i >= 4; i += 4) acc = add(acc, add(add(c[i], c[i + 1]), add(c[i + 2], c[i + 3])));
    for (; i < n; ++i) acc = add(acc, c[i]);
    return acc;
}

cam to_cam(const rt_camera *c)
{
    cam k;
    k.origin = mk(c->origin[0], c->origin[1], c->origin[2]);
    k.llc = mk(c->lower_left_corner[0], c->lower_left_corner[1], c->lower_left_corner[2]);
    k.hor = mk(c->horizontal[0], c->horizontal[1], c->horizontal[2]);
    k.ver = mk(c->vertical[0], c->vertical[1], c->vertical[2]);
    k.lens = c->lens_radius;
    k.corrected = c->mode == RT_CAMERA_CORRECTED;
    return k;
}

inline std::uint32_t rows_of(const rt_params &p)
{
    if (p.num_rows) return p.num_rows;
    std::uint32_t st = p.row_stride ? p.row_stride : 1;
    return p.row_offset >= p.height ? 0 : (p.height - p.row_offset + st - 1) / st;
}

// ---- the reference's CUDA variant, src/CUDA/cuda_impl.cu (RT_FLAG_CUDA_COMPAT) ----------
// Parity unpinned against the variant itself: it needs nvcc + thrust, absent here; this is a
// restatement from its source, line by line, with every binary32 op separately rounded.
struct xorshift32 {                                                             // cuda_impl.cu:13-41
    std::uint32_t s;
    float generate()
    {
        s ^= (s << 13);
        s ^= (s >> 17);
        s ^= (s << 5);
        return static_cast<float>(s) * (1.f / 4294967296.f);
    }
    v3 random_in_unit_sphere()                                                  // :43-56
    {
        v3 v;
        do {
            float x = generate() * 2.f - 1.f;
            float y = generate() * 2.f - 1.f;
            float z = generate() * 2.f - 1.f;
            v = mk(x, y, z);
        } while (length(v) > 1.f && s != 0u);  // a zero state never leaves 0: the variant would spin
        return v;
    }
};

// :131-186: shrinking t_max with strict comparisons; the lowest index wins a tie
inline hit cu_hit_world(const scene &sc, const ray &r)
{
    hit best{}; best.ok = false;
    float tmax = FLT_MAX;
    for (std::uint32_t i = 0; i < sc.n; ++i) {
        hit h;
        if (intersect(r, sc.s[i], .008f, tmax, h)) { best = h; tmax = h.t; }
    }
    return best;
}

// :288-324
inline v3 cu_color(const scene &sc, xorshift32 &g, ray r, std::uint32_t bounces, std::uint64_t &segments)
{
    v3 atten = mk(1.f, 1.f, 1.f);
    for (std::uint32_t b = 0; b < bounces; ++b) {
        ++segments;
        hit h = cu_hit_world(sc, r);
        if (!h.ok) return mulv(background(normalize(r.d).y * .5f + .5f), atten);   // :320
        const rt_material &m = sc.m[h.mat];
        v3 albedo = mk(m.albedo[0], m.albedo[1], m.albedo[2]);
        ray nr;
        bool valid = true;
        if (m.kind == RT_LAMBERT) {                                                // :197-206
            v3 rd = normalize(g.random_in_unit_sphere());
            nr = {h.p, add(h.n, rd)};
        } else if (m.kind == RT_METAL) {                                           // :208-222
            v3 refl = reflect(normalize(r.d), h.n);
            v3 rd = normalize(g.random_in_unit_sphere());
            nr = {h.p, add(refl, muls(rd, m.param))};
            valid = dot(nr.d, h.n) > 0.f;
        } else {                                                                   // :224-256
            v3 ud = normalize(r.d);
            v3 outward = neg(h.n);
            float ri = m.param;
            float cosv = dot(ud, h.n);
            if (cosv <= 0.f) {
                outward = muls(outward, -1.f);
                ri = 1.f / ri;
                cosv *= -1.f;
            }
            v3 refr = refract(ud, outward, ri);
            float prob = 1.f;
            if (length(refr) > 0.f) prob = schlick(ri, cosv);
            if (g.generate() < prob) nr = {h.p, reflect(ud, h.n)};
            else nr = {h.p, refr};
        }
        if (!valid) return mk(0.f, 0.f, 0.f);                                      // :308
        r = nr;
        atten = mulv(atten, albedo);                                               // :303-305
    }
    return mk(0.f, 0.f, 0.f);
}

} // namespace

extern "C" {

// cuda::data::render (:340-355) for every pixel of the rows of `params`; camera rays without a
// lens offset (camera.hxx:48-50); engine state = pixel index x + y W + seed (:408-413).
int oracle_render_cuda_compat(const rt_sphere *spheres, uint32_t n, const rt_material *mats, uint32_t nm,
                              const rt_camera *camera, const rt_params *params, int threads, float *out,
                              uint64_t *segments_out)
{
    if (!spheres || !mats || !camera || !params || !out || params->spp == 0) return RT_ERR_INVALID;
    const rt_params p = *params;
    const scene sc{spheres, n, mats, nm};
    const cam c = to_cam(camera);
    const std::uint32_t nrows = rows_of(p), stride = p.row_stride ? p.row_stride : 1;
    const bool full = p.flags & RT_FLAG_FULL_FRAME;
    if (threads < 1) threads = 1;
    std::vector<std::uint64_t> segs(threads, 0);
    auto worker = [&](int tid) {
        std::uint64_t seg = 0;
        for (std::uint32_t i = tid; i < nrows; i += threads) {
            const std::uint32_t y = p.row_offset + i * stride;
            for (std::uint32_t x = 0; x < p.width; ++x) {
                xorshift32 g{x + y * p.width + static_cast<std::uint32_t>(p.seed)};
                v3 col = mk(0.f, 0.f, 0.f);
                for (std::uint32_t s = 0; s < p.spp; ++s) {
                    float u = (static_cast<float>(x) + g.generate()) / static_cast<float>(p.width);
                    float v = (static_cast<float>(y) + g.generate()) / static_cast<float>(p.height);
                    ray r{c.origin, add(add(c.llc, muls(c.hor, u)), muls(c.ver, 1.f - v))};
                    col = add(col, cu_color(sc, g, r, p.max_depth, seg));
                }
                col = divs(col, static_cast<float>(p.spp));
                const std::size_t row = full ? y : i;
                float *o = out + (row * p.width + x) * 3;
                o[0] = col.x; o[1] = col.y; o[2] = col.z;
            }
        }
        segs[tid] = seg;
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
    worker(0);
    for (auto &t : pool) t.join();
    if (segments_out) {
        std::uint64_t s = 0;
        for (auto v : segs) s += v;
        *segments_out = s;
    }
    return RT_OK;
}

// Per-sample PCG streams (rng_mode 0, the GPU contract) or the reference's shared
// mt19937 streams (rng_mode 1; data seeded `seed`, camera `seed+1`, single thread).
int oracle_render_f32(const rt_sphere *spheres, uint32_t n, const rt_material *mats, uint32_t nm,
                      const rt_camera *camera, const rt_params *params, int rng_mode, int threads,
                      float *out, uint64_t *segments_out)
{
    if (!spheres || !mats || !camera || !params || !out || params->spp == 0) return RT_ERR_INVALID;
    const rt_params p = *params;
    const scene sc{spheres, n, mats, nm};
    const cam c = to_cam(camera);
    const std::uint32_t nrows = rows_of(p), stride = p.row_stride ? p.row_stride : 1;
    const bool full = p.flags & RT_FLAG_FULL_FRAME;
    if (rng_mode == 1) threads = 1;
    if (threads < 1) threads = 1;
    std::vector<std::uint64_t> segs(threads, 0);
    auto worker = [&](int tid) {
        std::vector<v3> samples(p.spp);
        pcg32 gd, gc;
        mt md, mc;
        md.g.seed(static_cast<std::uint32_t>(p.seed));
        mc.g.seed(static_cast<std::uint32_t>(p.seed + 1));
        std::uint64_t seg = 0;
        for (std::uint32_t i = tid; i < nrows; i += threads) {
            const std::uint32_t y = p.row_offset + i * stride;
            const float v = static_cast<float>(y) / static_cast<float>(p.height);  // main.cxx:192
            for (std::uint32_t x = 0; x < p.width; ++x) {
                const float u = static_cast<float>(x) / static_cast<float>(p.width); // main.cxx:195
                for (std::uint32_t s = 0; s < p.spp; ++s) {                          // main.cxx:197-203
                    if (rng_mode == 0) {
                        const std::uint64_t key = (static_cast<std::uint64_t>(y) * p.width + x) * p.spp + s;
                        gd.seed(key, 2u * p.seed);
                        gc.seed(key, 2u * p.seed + 1u);
                        float uu = u + canonical(gd) / static_cast<float>(p.width);
                        float vv = v + canonical(gd) / static_cast<float>(p.height);
                        samples[s] = color(sc, gd, camera_ray(c, gc, uu, vv), p.max_depth, seg);
                    } else {
                        float uu = u + canonical(md) / static_cast<float>(p.width);
                        float vv = v + canonical(md) / static_cast<float>(p.height);
                        samples[s] = color(sc, md, camera_ray(c, mc, uu, vv), p.max_depth, seg);
                    }
                }
                v3 col = divs(reduce_samples(samples), static_cast<float>(p.spp));  // main.cxx:205-207
                const std::size_t row = full ? y : i;
                float *o = out + (row * p.width + x) * 3;
                o[0] = col.x; o[1] = col.y; o[2] = col.z;
            }
        }
        segs[tid] = seg;
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
    worker(0);
    for (auto &t : pool) t.join();
    if (segments_out) {
        std::uint64_t s = 0;
        for (auto v : segs) s += v;
        *segments_out = s;
    }
    return RT_OK;
}

// app::gamma_correction + app::normalize_rgb_to_8bit (main.cxx:39-45, 77-85).
void oracle_epilogue_rgb8(const float *in, uint8_t *out, uint64_t n_values)
{
    const float g = 1.f / 2.2f;
    for (uint64_t i = 0; i < n_values; ++i) out[i] = static_cast<uint8_t>(255.f * std::pow(in[i], g));
}

// camera ctor, camera.hxx:24-44, with main.cxx:179-183's arguments available via
// oracle_camera_default.
int oracle_camera_init(const float pos[3], const float look[3], const float up[3], float aspect,
                       float vfov, float aperture, float focus, uint32_t mode, rt_camera *out)
{
    v3 P = mk(pos[0], pos[1], pos[2]), L = mk(look[0], look[1], look[2]), U = mk(up[0], up[1], up[2]);
    float theta = (vfov * static_cast<float>(0.01745329251994329576923690768489)) / 2.f;
    float h = std::tan(theta);
    float w = h * aspect;
    v3 W = normalize(sub(P, L));
    v3 Uu = normalize(cross(U, W));
    v3 V = normalize(cross(W, Uu));
    v3 llc = sub(P, muls(add(add(muls(Uu, w), muls(V, h)), W), focus));
    v3 hor = muls(muls(muls(Uu, w), focus), 2.f);
    v3 ver = muls(muls(muls(V, h), focus), 2.f);
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

int oracle_camera_default(uint32_t width, uint32_t height, uint32_t mode, rt_camera *out)
{
    const float pos[3] = {-4.f, 3.2f, 5.f}, look[3] = {0.f, 1.f, 0.f}, up[3] = {0.f, 1.f, 0.f};
    const float focus = length(sub(mk(pos[0], pos[1], pos[2]), mk(look[0], look[1], look[2])));
    return oracle_camera_init(pos, look, up, static_cast<float>(width) / static_cast<float>(height), 42.f,
                              0.0625f, focus, mode, out);
}

// ---- known-answer entry points (same record shapes as oracle/ref_harness.cpp) --------
// hit_world: rays[n][6] -> out[n][11] = {mat|0xffffffff, t, p[3], n[3]} as 32-bit words
void oracle_kat_hit(const rt_sphere *s, uint32_t ns, const rt_material *m, uint32_t nm, const float *rays,
                    uint32_t n, uint32_t *out, uint64_t *segments)
{
    scene sc{s, ns, m, nm};
    for (uint32_t i = 0; i < n; ++i) {
        ray r{mk(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), mk(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5])};
        hit h = hit_world(sc, r);
        float f[8] = {h.t, h.p.x, h.p.y, h.p.z, h.n.x, h.n.y, h.n.z, 0.f};
        if (!h.ok) std::memset(f, 0, sizeof f);
        out[8 * i] = h.ok ? h.mat : 0xffffffffu;
        std::memcpy(out + 8 * i + 1, f, 7 * 4);
    }
    if (segments) *segments = n;
}

// apply_material: in[n] = {mat, d[3], p[3], nrm[3], key} ; data stream seeded (key, 5).
// out[n] = {valid, o[3], d[3], atten[3], state_lo, state_hi}
void oracle_kat_scatter(const rt_material *m, uint32_t nm, const uint32_t *in, uint32_t n, uint32_t *out)
{
    scene sc{nullptr, 0, m, nm};
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t *r = in + 11 * i;
        float f[9];
        std::memcpy(f, r + 1, 36);
        hit h{mk(f[3], f[4], f[5]), mk(f[6], f[7], f[8]), 1.f, r[0], true};
        ray ray_in{mk(0.f, 0.f, 0.f), mk(f[0], f[1], f[2])};
        pcg32 g; g.seed(r[10], 5);
        ray o; v3 a;
        bool ok = apply_material(sc, g, ray_in, h, o, a);
        uint32_t *w = out + 12 * i;
        float res[9] = {o.o.x, o.o.y, o.o.z, o.d.x, o.d.y, o.d.z, a.x, a.y, a.z};
        if (!ok) std::memset(res, 0, sizeof res);
        w[0] = ok;
        std::memcpy(w + 1, res, 36);
        w[10] = static_cast<uint32_t>(g.state);
        w[11] = static_cast<uint32_t>(g.state >> 32);
    }
}

// camera.ray: in[n] = {u, v, key}; camera stream seeded (key, 3). out[n] = {o[3], d[3]}
void oracle_kat_camera(const rt_camera *camera, const uint32_t *in, uint32_t n, float *out)
{
    cam c = to_cam(camera);
    for (uint32_t i = 0; i < n; ++i) {
        float u, v;
        std::memcpy(&u, in + 3 * i, 4);
        std::memcpy(&v, in + 3 * i + 1, 4);
        pcg32 g; g.seed(in[3 * i + 2], 3);
        ray r = camera_ray(c, g, u, v);
        float *o = out + 6 * i;
        o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z; o[3] = r.d.x; o[4] = r.d.y; o[5] = r.d.z;
    }
}

// misc: in[n] = {t, c[3], I[3], N[3], eta, cos}; out[n] = {bg[3], gamma[3], u8[3], refract[3], reflect[3], schlick}
void oracle_kat_misc(const float *in, uint32_t n, uint32_t *out)
{
    for (uint32_t i = 0; i < n; ++i) {
        const float *r = in + 12 * i;
        v3 bg = background(r[0]);
        v3 c = mk(r[1], r[2], r[3]);
        const float g = 1.f / 2.2f;
        v3 gm = mk(std::pow(c.x, g), std::pow(c.y, g), std::pow(c.z, g));
        v3 I = mk(r[4], r[5], r[6]), N = mk(r[7], r[8], r[9]);
        v3 rf = refract(I, N, r[10]);
        v3 rl = reflect(I, N);
        float sc = schlick(r[10], r[11]);
        uint32_t *w = out + 16 * i;
        float f1[6] = {bg.x, bg.y, bg.z, gm.x, gm.y, gm.z};
        std::memcpy(w, f1, 24);
        w[6] = static_cast<uint8_t>(255.f * gm.x);
        w[7] = static_cast<uint8_t>(255.f * gm.y);
        w[8] = static_cast<uint8_t>(255.f * gm.z);
        float f2[7] = {rf.x, rf.y, rf.z, rl.x, rl.y, rl.z, sc};
        std::memcpy(w + 9, f2, 28);
    }
}

} // extern "C"
