// rt_render_impl.hpp — header-only C++ drop-in for the reference's accelerated render entry.
//
// The reference declares and calls
//     extern void cuda_impl(std::uint32_t width, std::uint32_t height,
//                           std::vector<math::u8vec3> &image_texels);   // src/main.cxx:18, :114
// This header provides the same shape on top of the C ABI (rt_api.h), plus a form that takes
// the reference's own scene object (raytracer::data, src/raytracer.hxx:19-30) so the CPU render
// loop of src/main.cxx:185-215 can be replaced with one call. Like cuda_impl (cuda_impl.cu:101-114)
// failures throw std::runtime_error; the C ABI underneath never throws.
//
// Texel is any 3-byte RGB type (math::u8vec3); the scene types are duck-typed:
//   spheres:   .center.{x,y,z}, .radius, .material_index        (primitives::sphere)
//   materials: std::variant-like visited with std::visit, alternatives exposing .albedo.{x,y,z}
//              and .roughness (metal) / .refraction_index (dielectric) (material.hxx)
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <variant>
#include <vector>

#include "rt_api.h"

namespace rt {

inline void check(int status, const char *what)
{
    if (status != RT_OK) throw std::runtime_error(std::string(what) + ": " + rt_last_error());
}

// The reference's render settings: spp = app::data::sampling_number (main.cxx:23),
// depth = raytracer::data::bounces_number (raytracer.hxx:20).
struct settings {
    std::uint32_t spp = 16;
    std::uint32_t max_depth = 64;
    std::uint64_t seed = 1234;
    std::uint32_t camera_mode = RT_CAMERA_REFERENCE;
    std::uint32_t flags = 0;  // RT_FLAG_FAST_MATH for the tolerance-bounded kernel
};

template <class Texel>
void render_rgb8(const std::vector<rt_sphere> &spheres, const std::vector<rt_material> &materials,
                 const rt_camera &camera, std::uint32_t width, std::uint32_t height, const settings &s,
                 std::vector<Texel> &image_texels)
{
    static_assert(sizeof(Texel) == 3, "Texel must be a packed 3 x uint8 RGB type (math::u8vec3)");
    image_texels.resize(static_cast<std::size_t>(width) * height);
    rt_params p{width, height, s.spp, s.max_depth, s.seed, 0, 1, 0, s.flags};
    check(rt_render_rgb8(spheres.data(), static_cast<std::uint32_t>(spheres.size()), materials.data(),
                         static_cast<std::uint32_t>(materials.size()), &camera, &p,
                         reinterpret_cast<std::uint8_t *>(image_texels.data()), nullptr),
          "rt_render_rgb8");
}

// Converts the reference's raytracer::data (or anything shaped like it). Needs C++20 (the
// reference builds as C++20, CMakeLists.txt:32).
template <class RaytracerData>
void pack_scene(const RaytracerData &data, std::vector<rt_sphere> &spheres, std::vector<rt_material> &materials)
{
    spheres.clear();
    materials.clear();
    for (const auto &sp : data.spheres)
        spheres.push_back({{sp.center.x, sp.center.y, sp.center.z}, sp.radius,
                           static_cast<std::uint32_t>(sp.material_index)});
    for (const auto &mt : data.materials) {
        rt_material r{};
        std::visit([&](const auto &m) {
            using T = std::decay_t<decltype(m)>;
            r.albedo[0] = m.albedo.x; r.albedo[1] = m.albedo.y; r.albedo[2] = m.albedo.z;
            if constexpr (requires(const T &x) { x.roughness; }) { r.kind = RT_METAL; r.param = m.roughness; }
            else if constexpr (requires(const T &x) { x.refraction_index; }) { r.kind = RT_DIELECTRIC; r.param = m.refraction_index; }
            else { r.kind = RT_LAMBERT; r.param = 0.f; }
        }, mt);
        materials.push_back(r);
    }
}

// Replacement for the CPU render loop of main.cxx:185-215 given the reference's scene: the
// camera is the one main() builds (main.cxx:179-183).
template <class RaytracerData, class Texel>
void render_impl(const RaytracerData &data, std::uint32_t width, std::uint32_t height, std::vector<Texel> &image_texels,
                 const settings &s = {})
{
    std::vector<rt_sphere> spheres;
    std::vector<rt_material> materials;
    pack_scene(data, spheres, materials);
    rt_camera cam;
    check(rt_camera_default(width, height, s.camera_mode, &cam), "rt_camera_default");
    render_rgb8(spheres, materials, cam, width, height, s, image_texels);
}

// The literal cuda_impl shape (main.cxx:18): scene of main.cxx:120-129, camera of :179-183.
template <class Texel>
void render_impl(std::uint32_t width, std::uint32_t height, std::vector<Texel> &image_texels, const settings &s = {})
{
    std::uint32_t ns = 0, nm = 0;
    check(rt_scene_simple(nullptr, 0, &ns, nullptr, 0, &nm), "rt_scene_simple");
    std::vector<rt_sphere> spheres(ns);
    std::vector<rt_material> materials(nm);
    check(rt_scene_simple(spheres.data(), ns, &ns, materials.data(), nm, &nm), "rt_scene_simple");
    rt_camera cam;
    check(rt_camera_default(width, height, s.camera_mode, &cam), "rt_camera_default");
    render_rgb8(spheres, materials, cam, width, height, s, image_texels);
}

// The CUDA variant itself, src/CUDA/cuda_impl.cu:384-453, under its own name and shape: its
// scene (:425-437), camera (:371-375), 48 spp, 32 bounces, one xorshift32 engine per pixel
// (RT_FLAG_CUDA_COMPAT). In the reference tree:
//     void cuda_impl(std::uint32_t w, std::uint32_t h, std::vector<math::u8vec3> &t) { rt::cuda_impl(w, h, t); }
template <class Texel>
void cuda_impl(std::uint32_t width, std::uint32_t height, std::vector<Texel> &image_texels)
{
    static_assert(sizeof(Texel) == 3, "Texel must be a packed 3 x uint8 RGB type (math::u8vec3)");
    image_texels.resize(static_cast<std::size_t>(width) * height);
    check(rt_render_cuda_impl(width, height, reinterpret_cast<std::uint8_t *>(image_texels.data())),
          "rt_render_cuda_impl");
}

// The synchronous calls above keep one context per device between calls (the scene's device
// copy, streams, workspaces), so that a frame per call costs the frame. Frees it
// (process exit does too).
inline void release_cached() { check(rt_release_cached(), "rt_release_cached"); }

} // namespace rt
