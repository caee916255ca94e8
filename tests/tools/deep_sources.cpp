// TEST INFRASTRUCTURE (analysis only): where do the deep paths of a frame come from?
// Builds on the CPU restatement (oracle/rt_oracle.cpp, included) and traces every sample of
// the given rows like oracle_render_f32 (rng_mode 0, the GPU contract), recording per sample
// its segment count, the kind of its primary hit and the segment of its first dielectric hit.
// Used by tests/tools/deep_sources.py for DESIGN.md §4.7 (the dealing order of a lone pass).
#include "../../oracle/rt_oracle.cpp"

namespace {
// app::color (main.cxx:52-75) with a trace: returns the segment count; prim = kind of the
// primary hit (0 sky, 1 lambert, 2 metal, 3 dielectric), fdi = segment (1-based) of the first
// dielectric hit or 0; ground = a lambert hit below y = -0.05 (the huge scene's ground, top at y = -0.125)
template <class G>
std::uint32_t color_trace(const scene &sc, G &g, ray r, std::uint32_t depth, std::uint32_t &prim, std::uint32_t &fdi)
{
    prim = 0;
    fdi = 0;
    std::uint32_t seg = 0;
    for (std::uint32_t b = 0; b < depth; ++b) {
        ++seg;
        hit h = hit_world(sc, r);
        if (!h.ok) return seg;
        const std::uint32_t kind = sc.m[h.mat].kind;
        if (b == 0) prim = kind + 1 + (kind == RT_LAMBERT && h.p.y < -0.05f ? 3u : 0u);
        if (kind == RT_DIELECTRIC && !fdi) fdi = seg;
        ray nr; v3 e;
        if (!apply_material(sc, g, r, h, nr, e)) return seg;
        r = nr;
    }
    return seg;
}
} // namespace

extern "C" int deep_sources(const rt_sphere *spheres, uint32_t n, const rt_material *mats, uint32_t nm,
                            const rt_camera *camera, const rt_params *params, int threads,
                            uint32_t *segs_out /* [rows][W][spp] */, uint8_t *prim_out, uint8_t *fdi_out)
{
    const rt_params p = *params;
    const scene sc{spheres, n, mats, nm};
    const cam c = to_cam(camera);
    const std::uint32_t nrows = rows_of(p), stride = p.row_stride ? p.row_stride : 1;
    auto worker = [&](int tid) {
        pcg32 gd, gc;
        for (std::uint32_t i = tid; i < nrows; i += threads) {
            const std::uint32_t y = p.row_offset + i * stride;
            const float v = static_cast<float>(y) / static_cast<float>(p.height);
            for (std::uint32_t x = 0; x < p.width; ++x) {
                const float u = static_cast<float>(x) / static_cast<float>(p.width);
                for (std::uint32_t s = 0; s < p.spp; ++s) {
                    const std::uint64_t key = (static_cast<std::uint64_t>(y) * p.width + x) * p.spp + s;
                    gd.seed(key, 2u * p.seed);
                    gc.seed(key, 2u * p.seed + 1u);
                    float uu = u + canonical(gd) / static_cast<float>(p.width);
                    float vv = v + canonical(gd) / static_cast<float>(p.height);
                    std::uint32_t pr, fd;
                    const std::uint32_t sg = color_trace(sc, gd, camera_ray(c, gc, uu, vv), p.max_depth, pr, fd);
                    const std::size_t o = (static_cast<std::size_t>(i) * p.width + x) * p.spp + s;
                    segs_out[o] = sg;
                    prim_out[o] = static_cast<std::uint8_t>(pr);
                    fdi_out[o] = static_cast<std::uint8_t>(std::min<std::uint32_t>(fd, 255u));
                }
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
    worker(0);
    for (auto &t : pool) t.join();
    return RT_OK;
}
