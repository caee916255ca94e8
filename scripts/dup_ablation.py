#!/usr/bin/env python3
"""Timing-only builds (wrong nothing: same paths, same bits) that run one part of the render
loop twice on an opaque copy of its inputs, so the frame-time difference is that part's marginal
cost.  python scripts/dup_ablation.py  ->  scripts/_abl/dup_<part>/librt_mi355x.so"""
import os
import shutil
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "raytracinginoneweekend_amd", "csrc")
K = "rt_kernel.hip"
PATCHES = {
    "reject": ("            const f3 r = random_in_unit_sphere_capped<STATS>(st, inc, got, dbg);\n",
               "            {\n"
               "                uint64_t st2 = st;\n"
               "                uint32_t lo2 = (uint32_t)st2, hi2 = (uint32_t)(st2 >> 32);\n"
               "                asm volatile(\"\" : \"+v\"(lo2), \"+v\"(hi2));\n"
               "                st2 = ((uint64_t)hi2 << 32) | lo2;\n"
               "                bool g2;\n"
               "                const f3 r2 = random_in_unit_sphere_capped<STATS>(st2, inc, g2, dbg);\n"
               "                asm volatile(\"\" ::\"v\"(r2.x), \"v\"(r2.y), \"v\"(r2.z), \"v\"((uint32_t)st2), \"v\"((uint32_t)g2));\n"
               "            }\n"),
    "hit": ("            h = closest_hit<FAST, CULL, STATS, COUNT>(P, geo, sidx, clus, o, d, rd, dbg, wt, walk, wm, tw, key0);\n",
            "            {\n"
            "                f3 o2 = o;\n"
            "                asm volatile(\"\" : \"+v\"(o2.x));\n"
            "                const Hit h2 = closest_hit<FAST, CULL, STATS, COUNT>(P, geo, sidx, clus, o2, d, rd, dbg, wt, walk, wm, tw, key0);\n"
            "                asm volatile(\"\" ::\"v\"((uint32_t)h2.key), \"v\"((uint32_t)(h2.key >> 32)));\n"
            "            }\n"),
    "boxes2": ("            const bool bs = box_pass(rb, s0, s1, t_lo, h.t() * 1.002f);\n",
               "            {\n"
               "                float4 s0b = s0;\n"
               "                asm volatile(\"\" : \"+v\"(s0b.x));\n"
               "                const bool bs2 = box_pass(rb, s0b, s1, t_lo, h.t() * 1.002f);\n"
               "                asm volatile(\"\" ::\"v\"((uint32_t)bs2));\n"
               "            }\n"),
    "ground": ("    if (RT_GROUND1 && p.n_always == 1u) test_block8<FAST, STATS, 1>(geo, sidx, 0, o, d, rd, h, dbg);\n",
               "    {\n"
               "        f3 o2 = o;\n"
               "        asm volatile(\"\" : \"+v\"(o2.x));\n"
               "        Hit h2{key0};\n"
               "        test_block8<FAST, STATS, 1>(geo, sidx, 0, o2, d, rd, h2, dbg);\n"
               "        asm volatile(\"\" ::\"v\"((uint32_t)h2.key), \"v\"((uint32_t)(h2.key >> 32)));\n"
               "    }\n"),
}
PATCHES.update({
    "members_t": ("        members_transposed<FAST, STATS>(geo, sidx, start, cnt, M, req, tw, o, d, rd, h, dbg);\n",
                  "        {\n"
                  "            f3 o2 = o;\n"
                  "            asm volatile(\"\" : \"+v\"(o2.x));\n"
                  "            Hit h2 = h;\n"
                  "            members_transposed<FAST, STATS>(geo, sidx, start, cnt, M, req, tw, o2, d, rd, h2, dbg);\n"
                  "            asm volatile(\"\" ::\"v\"((uint32_t)h2.key), \"v\"((uint32_t)(h2.key >> 32)));\n"
                  "        }\n"),
    "members_l": ("        run_members<FAST, STATS>(geo, sidx, start, cnt, o, d, rd, h, dbg);\n",
                  "        {\n"
                  "            f3 o2 = o;\n"
                  "            asm volatile(\"\" : \"+v\"(o2.x));\n"
                  "            Hit h2 = h;\n"
                  "            run_members<FAST, STATS>(geo, sidx, start, cnt, o2, d, rd, h2, dbg);\n"
                  "            asm volatile(\"\" ::\"v\"((uint32_t)h2.key), \"v\"((uint32_t)(h2.key >> 32)));\n"
                  "        }\n"),
    "refract": ("                            const f3 refr = refract(ud, outward, ri);\n",
                "                            {\n"
                "                                f3 u2 = ud;\n"
                "                                asm volatile(\"\" : \"+v\"(u2.x));\n"
                "                                const f3 r2 = refract(u2, outward, ri);\n"
                "                                const float p2 = schlick_x(xs, cosv + u2.x * 0.f);\n"
                "                                asm volatile(\"\" ::\"v\"(r2.x), \"v\"(r2.y), \"v\"(r2.z), \"v\"(p2));\n"
                "                            }\n"),
    # the fresh sample start: item -> pixel, sample, key, seeds, two jitter draws, uu vv
    "start": ("            att = mk(1.f, 1.f, 1.f);\n            depth = 0;\n",
              "            {\n"
              "                uint32_t it2 = it;\n"
              "                asm volatile(\"\" : \"+v\"(it2));\n"
              "                const uint32_t sl2 = it2 & kItSlot;\n"
              "                const bool pr2 = sl2 < P.n_pair_items;\n"
              "                const uint32_t J2 = pr2 ? sl2 : sl2 - P.n_pair_items;\n"
              "                const uint32_t q2 = udiv(J2, fc->div_n_pixels);\n"
              "                const uint32_t ls2 = pr2 ? 2u * q2 + (it2 >> 31) : 2u * fc->n_pairs + q2;\n"
              "                uint32_t px2, rr2;\n"
              "                pixel_of(*fc, J2 - q2 * fc->n_pixels, px2, rr2);\n"
              "                const uint32_t py2 = fc->row_offset + rr2 * fc->row_stride;\n"
              "                const uint64_t key2 = (uint64_t)(py2 * fc->W + px2) * fc->spp + fc->sample_begin + ls2;\n"
              "                uint64_t rng2 = key2 * kPcgMul + inc_data * (kPcgMul + 1u);\n"
              "                const float xu2 = canonical(rng2, inc_data);\n"
              "                const float xv2 = canonical(rng2, inc_data);\n"
              "                const float uu2 = div_const((float)px2, fc->fW, fc->rW, true) + div_const(xu2, fc->fW, fc->rW, true);\n"
              "                const float vv2 = div_const((float)py2, fc->fH, fc->rH, true) + div_const(xv2, fc->fH, fc->rH, true);\n"
              "                asm volatile(\"\" ::\"v\"(uu2), \"v\"(vv2), \"v\"((uint32_t)rng2));\n"
              "            }\n"),
    # hit shading for metal/dielectric lanes: hit point, normal, unit direction, reflection
    "shade": ("                        const f3 rf = reflect(ud, hn);\n",
              "                        {\n"
              "                            f3 d2 = d;\n"
              "                            asm volatile(\"\" : \"+v\"(d2.x));\n"
              "                            const f3 dv2 = (o + d2 * t) - ctr;\n"
              "                            const f3 hn2 = (P.fast_roots && all_lanes_min_abs_ok(dv2)) ? div3_short(dv2, sf.w) : dv2 / sf.w;\n"
              "                            const f3 ud2 = (rd.fd != 0u && all_lanes_min_abs_ok(d2)) ? div3_short(d2, sqrt_scaled(a)) : normalize(d2);\n"
              "                            const f3 rf2 = reflect(ud2, hn2);\n"
              "                            asm volatile(\"\" ::\"v\"(rf2.x), \"v\"(rf2.y), \"v\"(rf2.z));\n"
              "                        }\n"),
})
ONLY = os.environ.get("DUP_ONLY", "").split(",") if os.environ.get("DUP_ONLY") else None
FLAGS = ["-std=c++17", "-O3", "-fno-slp-vectorize", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
         "-fPIC"]
for name, (anchor, extra) in PATCHES.items():
    if ONLY and name not in ONLY:
        continue
    out = os.path.join(REPO, "scripts", "_abl", "dup_" + name)
    src = os.path.join(out, "src")
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(src)
    for f in ("rt_kernel.hip", "rt_device.h", "rt_consts.h"):
        shutil.copy(os.path.join(SRC, f), src)
    os.makedirs(os.path.join(out, "include"), exist_ok=True)
    text = open(os.path.join(src, K)).read()
    assert text.count(anchor) >= 1, name
    # the render loop's copy (the first occurrence; the wavefront kernel has its own)
    text = text.replace(anchor, anchor + extra if name != "ground" else extra + anchor, 1)
    open(os.path.join(src, K), "w").write(text)
    inc = ["-I", os.path.join(REPO, "include")]
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *inc, "-Rpass-analysis=kernel-resource-usage", "-c",
                        os.path.join(src, K), "-o", os.path.join(out, "k.o")], check=True, capture_output=True, text=True)
    lines = r.stderr.splitlines()
    i = next(j for j, line in enumerate(lines) if "render_kernelILi0ELi7ELb0ELb0E" in line)
    print(name, " ".join(x.split(":")[-1].strip().split(" [")[0] for x in lines[i + 1:i + 9]
                         if "GPRs" in x or "Occupancy" in x))
    # the host side is unchanged: the product build's object (make -C raytracinginoneweekend_amd/csrc)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(out, "librt_mi355x.so"), os.path.join(out, "k.o"), os.path.join(SRC, "_obj", "rt_host.o"),
                    os.path.join(SRC, "_obj", "rt_host_build.o"), "-Wl,--no-undefined"], check=True)
    shutil.rmtree(src)
    print("built", out)
