// Example: the reference's main() with its CPU render loop (src/main.cxx:185-215) replaced by
// one call into librt_mi355x.so through include/rt_render_impl.hpp. The scene types below are
// this example's own minimal stand-ins shaped like primitives::sphere / material::* /
// raytracer::data so the example builds without the reference; in the reference tree the real
// types are used unchanged.
//   g++ -std=c++20 -Iinclude examples/dropin_main.cpp -Lraytracinginoneweekend_amd -lrt_mi355x
//       -Wl,-rpath,$PWD/raytracinginoneweekend_amd -o dropin && ./dropin out.ppm [spp | cuda]
// With "cuda" it calls rt::cuda_impl, the CUDA variant's own scene and semantics.
#include <cstdio>
#include <fstream>
#include <string>
#include <variant>
#include <vector>

#include "rt_render_impl.hpp"

namespace ex {
struct vec3 { float x, y, z; };
struct u8vec3 { std::uint8_t x, y, z; };
struct lambert { vec3 albedo; };
struct metal { vec3 albedo; float roughness; };
struct dielectric { vec3 albedo; float refraction_index; };
struct sphere { vec3 center; float radius; std::size_t material_index; };
struct data { std::vector<sphere> spheres; std::vector<std::variant<lambert, metal, dielectric>> materials; };
}  // namespace ex

int main(int argc, char **argv)
{
    const std::uint32_t W = 200, H = 100;
    ex::data d;  // src/main.cxx:120-129
    d.materials.push_back(ex::lambert{{.1f, .2f, .5f}});
    d.materials.push_back(ex::metal{{.8f, .6f, .2f}, 0.f});
    d.materials.push_back(ex::dielectric{{1.f, 1.f, 1.f}, 1.5f});
    d.materials.push_back(ex::lambert{{.64f, .8f, .0f}});
    d.spheres.push_back({{0, 1, 0}, 1.f, 0});
    d.spheres.push_back({{0, -1000.125f, 0}, 1000.f, 3});
    d.spheres.push_back({{+2, 1, 0}, 1.f, 1});
    d.spheres.push_back({{-2, 1, 0}, 1.f, 2});
    d.spheres.push_back({{-2, 1, 0}, -.99f, 2});
    std::vector<ex::u8vec3> texels;
    try {
        if (argc > 2 && std::string(argv[2]) == "cuda") {
            rt::cuda_impl(W, H, texels);  // was: cuda_impl(app_data.width, app_data.height, output)
        } else {
            rt::settings s;
            s.spp = argc > 2 ? static_cast<std::uint32_t>(std::atoi(argv[2])) : 16u;
            rt::render_impl(d, W, H, texels, s);
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "render failed: %s\n", e.what());
        return 3;
    }
    // app::save_to_file (src/main.cxx:87-101)
    std::ofstream f(argc > 1 ? argv[1] : "image.ppm", std::ios::binary);
    f << "P6\n" << W << " " << H << "\n255\n";
    f.write(reinterpret_cast<const char *>(texels.data()), texels.size() * 3);
    return 0;
}
