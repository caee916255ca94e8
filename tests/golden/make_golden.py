#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs oracle/_ref/ref_harness_{pcg,mt} — the reference's own CPU render path built by
oracle/build_ref.sh from /root/reference (this container only) — and stores inputs and
outputs as small binary files plus manifest.json. Nothing of the reference's source is
stored: the fixtures are data (scene records, f32/u8 framebuffers, known-answer tables).

    python tests/golden/make_golden.py          # needs /root/reference
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref")

# (name, harness args, kind). Renders use the per-sample PCG engine (the GPU contract)
# unless marked "mt" (the reference's verbatim shared mt19937 streams).
RENDERS = [
    # config 1: simple scene 200x100 @1spp (the reference's CPU case)
    ("c1_simple_200x100_s1", ["--scene", "simple", "--w", "200", "--h", "100", "--spp", "1"], "pcg"),
    ("c1_simple_200x100_s1_mt", ["--scene", "simple", "--w", "200", "--h", "100", "--spp", "1"], "mt"),
    ("simple_64x32_s4_corr_d50", ["--scene", "simple", "--w", "64", "--h", "32", "--spp", "4",
                                  "--camera", "corrected", "--depth", "50"], "pcg"),
    ("simple_48x24_s7_corr", ["--scene", "simple", "--w", "48", "--h", "24", "--spp", "7",
                              "--camera", "corrected"], "pcg"),
    ("huge_64x36_s4", ["--scene", "@huge", "--w", "64", "--h", "36", "--spp", "4"], "pcg"),
    ("huge_48x27_s2_corr", ["--scene", "@huge", "--w", "48", "--h", "27", "--spp", "2",
                            "--camera", "corrected"], "pcg"),
    # full-size config 3 geometry, two rows (y = 100, 460) of 1280x720 @2spp
    ("huge_1280x720_rows100+360_s2", ["--scene", "@huge", "--w", "1280", "--h", "720", "--spp", "2",
                                      "--row0", "100", "--row-step", "360", "--rows", "2"], "pcg"),
    ("huge_1280x720_row300_s2_corr", ["--scene", "@huge", "--w", "1280", "--h", "720", "--spp", "2",
                                      "--row0", "300", "--rows", "1", "--camera", "corrected"], "pcg"),
    # one full-spp row of config 4 (3840x2160 @256spp; 13 render passes on one GPU) and of
    # config 5 (1280x720 @1024spp; 6 passes): the multi-pass frames checked against the reference
    ("c4_huge_3840x2160_row1133_s256", ["--scene", "@huge", "--w", "3840", "--h", "2160", "--spp", "256",
                                        "--row0", "1133", "--rows", "1"], "pcg"),
    ("c5_huge_1280x720_row377_s1024", ["--scene", "@huge", "--w", "1280", "--h", "720", "--spp", "1024",
                                       "--row0", "377", "--rows", "1"], "pcg"),
]
# renders whose u8 frame is also written by the reference's own PPM writer (app::save_to_file)
PPM = {"c1_simple_200x100_s1"}
KATS = [("kat_hit", "hit", "@huge", 2048), ("kat_scatter", "scatter", "@huge", 2048),
        ("kat_camera", "camera", "simple", 512), ("kat_misc", "misc", "simple", 1024)]


def sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    if not os.path.exists(os.path.join(REF, "ref_harness_pcg")):
        subprocess.run(["bash", os.path.join(REPO, "oracle", "build_ref.sh")], check=True)
    pcg, mt = os.path.join(REF, "ref_harness_pcg"), os.path.join(REF, "ref_harness_mt")
    manifest = {"generator": "oracle/_ref/ref_harness_* (reference CPU path, oracle/build_ref.sh)",
                "rng": {"pcg": "per-sample PCG32: data seq 2*seed, camera seq 2*seed+1, key=(y*W+x)*spp+s",
                        "mt": "reference std::mt19937 streams, data seed=seed, camera seed=seed+1"},
                "seed": 1234, "scenes": {}, "renders": {}, "kats": {}}
    huge = os.path.join(HERE, "scene_huge_1234.bin")
    simple = os.path.join(HERE, "scene_simple.bin")
    subprocess.run([pcg, "--scene", "huge", "--scene-seed", "1234", "--dump-scene", huge,
                    "--w", "1", "--h", "1"], check=True)
    subprocess.run([pcg, "--scene", "simple", "--dump-scene", simple, "--w", "1", "--h", "1"], check=True)
    manifest["scenes"]["huge"] = {"file": "scene_huge_1234.bin", "seed": 1234, "sha256": sha(huge)}
    manifest["scenes"]["simple"] = {"file": "scene_simple.bin", "sha256": sha(simple)}
    for name, args, kind in RENDERS:
        args = [huge if a == "@huge" else a for a in args]
        f32 = os.path.join(HERE, name + ".f32")
        u8 = os.path.join(HERE, name + ".u8")
        exe = pcg if kind == "pcg" else mt
        ppm = os.path.join(HERE, name + ".ppm") if name in PPM else None
        subprocess.run([exe] + args + ["--seed", "1234", "--threads", "8", "--out-f32", f32,
                                       "--out-u8", u8] + (["--out-ppm", ppm] if ppm else []), check=True)
        a = dict(zip(args[::2], args[1::2]))
        scene = "huge" if a["--scene"] == huge else "simple"
        W, H = int(a["--w"]), int(a["--h"])
        row0, step = int(a.get("--row0", 0)), int(a.get("--row-step", 1))
        rows = int(a.get("--rows", (H - row0 + step - 1) // step))
        manifest["renders"][name] = {
            "scene": scene, "width": W, "height": H, "spp": int(a["--spp"]),
            "depth": int(a.get("--depth", 64)), "camera": a.get("--camera", "reference"),
            "row_offset": row0, "row_stride": step, "num_rows": rows, "rng": kind, "seed": 1234,
            "f32": name + ".f32", "u8": name + ".u8", "sha256_f32": sha(f32), "sha256_u8": sha(u8)}
        if ppm:
            manifest["renders"][name].update({"ppm": name + ".ppm", "sha256_ppm": sha(ppm)})
    for name, kat, scene, n in KATS:
        out = os.path.join(HERE, name + ".bin")
        sc = huge if scene == "@huge" else scene
        subprocess.run([pcg, "--scene", sc, "--kat", kat, "--kat-n", str(n), "--kat-out", out,
                        "--w", "200", "--h", "100"], check=True)
        manifest["kats"][kat] = {"file": name + ".bin", "n": n, "scene": "huge" if scene == "@huge" else scene,
                                 "camera_w": 200, "camera_h": 100, "sha256": sha(out)}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    total = sum(os.path.getsize(os.path.join(HERE, p)) for p in os.listdir(HERE))
    print(f"golden fixtures written: {total/1e6:.2f} MB")


if __name__ == "__main__":
    sys.exit(main())
