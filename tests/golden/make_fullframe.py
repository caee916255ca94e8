#!/usr/bin/env python3
"""Whole-frame digests of BASELINE configs 2-5 from the REFERENCE itself (this container only).

Runs oracle/_ref/ref_harness_pcg — the reference's own CPU render path (src/main.cxx:185-215,
raytracer.hxx, built by oracle/build_ref.sh) with the per-sample PCG32 engine of the GPU
contract — on each config's FULL frame and stores, in tests/golden/fullframe.json:
  * sha256 of the whole f32 frame (linear, pre-gamma, main.cxx:205-207) and of the u8 frame
    (gamma + normalize_rgb_to_8bit, main.cxx:39-45,77-85);
  * a 64-bit prefix of the sha256 of every f32 row, so a GPU mismatch names its rows;
  * per-channel sums of the f32 frame (a size-independent property, float64).
The frames themselves (11-100 MB) are not committed: they are data the tests re-derive
on the GPU and compare by digest.

    python tests/golden/make_fullframe.py [c2 c3 c5 c4]     # needs /root/reference (build_ref.sh)
    python tests/golden/make_fullframe.py --dropin

--dropin: the frame the reference's own main() renders in its debug build (src/main.cxx:23-27:
512x256, 16 spp, simple scene, depth 64), written by the reference's app::save_to_file
(main.cxx:87-101) to dropin_simple_512x256_s16.ppm, with its digests in dropin.json — what
examples/_ref/ref_main_dropin (the reference's main() with the INTEGRATION.md swap,
examples/build_ref_dropin.sh) must reproduce on the GPU.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
EXE = os.path.join(REPO, "oracle", "_ref", "ref_harness_pcg")
OUT = os.path.join(HERE, "fullframe.json")

# name: (scene, W, H, spp, depth) — BASELINE.json configs, reference camera, seed 1234
CONFIGS = {
    "c2": ("simple", 1280, 720, 64, 50),
    "c3": ("huge", 1280, 720, 128, 64),
    "c5": ("huge", 1280, 720, 1024, 64),
    "c4": ("huge", 3840, 2160, 256, 64),
}


def dropin():
    W, H, spp = 512, 256, 16
    ppm = os.path.join(HERE, "dropin_simple_512x256_s16.ppm")
    with tempfile.TemporaryDirectory() as td:
        f32p, u8p = os.path.join(td, "f.f32"), os.path.join(td, "f.u8")
        subprocess.run([EXE, "--scene", "simple", "--w", str(W), "--h", str(H), "--spp", str(spp), "--depth", "64",
                        "--seed", "1234", "--camera", "reference", "--threads", str(os.cpu_count() or 8),
                        "--out-f32", f32p, "--out-u8", u8p, "--out-ppm", ppm], check=True)
        f32 = open(f32p, "rb").read()
        u8 = open(u8p, "rb").read()
    rec = {"scene": "simple", "width": W, "height": H, "spp": spp, "depth": 64, "camera": "reference", "seed": 1234,
           "rng": "pcg", "ppm": os.path.basename(ppm), "sha256_ppm": hashlib.sha256(open(ppm, "rb").read()).hexdigest(),
           "sha256_f32": hashlib.sha256(f32).hexdigest(), "sha256_u8": hashlib.sha256(u8).hexdigest(),
           "generator": "oracle/_ref/ref_harness_pcg --out-ppm (the reference's app::save_to_file)"}
    with open(os.path.join(HERE, "dropin.json"), "w") as f:
        json.dump(rec, f, indent=1, sort_keys=True)
    print("dropin:", rec["sha256_ppm"][:16])


def main(argv):
    if argv == ["--dropin"]:
        return dropin()
    names = argv or ["c2", "c3", "c5", "c4"]
    threads = str(os.cpu_count() or 8)
    rec = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            rec = json.load(f)
    huge = os.path.join(HERE, "scene_huge_1234.bin")
    for name in names:
        scene, W, H, spp, depth = CONFIGS[name]
        with tempfile.TemporaryDirectory() as td:
            f32p, u8p = os.path.join(td, "f.f32"), os.path.join(td, "f.u8")
            cmd = [EXE, "--scene", huge if scene == "huge" else "simple", "--w", str(W), "--h", str(H),
                   "--spp", str(spp), "--depth", str(depth), "--seed", "1234", "--camera", "reference",
                   "--threads", threads, "--out-f32", f32p, "--out-u8", u8p]
            t0 = time.time()
            subprocess.run(cmd, check=True)
            sec = time.time() - t0
            f32 = np.fromfile(f32p, dtype=np.float32).reshape(H, W, 3)
            u8 = np.fromfile(u8p, dtype=np.uint8)
        rows = [hashlib.sha256(f32[y].tobytes()).hexdigest()[:16] for y in range(H)]
        rec[name] = {
            "scene": scene, "width": W, "height": H, "spp": spp, "depth": depth, "camera": "reference",
            "seed": 1234, "rng": "pcg", "generator": "oracle/_ref/ref_harness_pcg (reference CPU path)",
            "sha256_f32": hashlib.sha256(f32.tobytes()).hexdigest(),
            "sha256_u8": hashlib.sha256(u8.tobytes()).hexdigest(),
            "channel_sums": [float(x) for x in f32.astype(np.float64).sum(axis=(0, 1))],
            "row_sha256_16": rows, "cpu_seconds_wall": round(sec, 1), "cpu_threads": int(threads)}
        with open(OUT, "w") as f:
            json.dump(rec, f, indent=0, sort_keys=True)
        print(f"{name}: {W}x{H}@{spp} depth {depth} in {sec:.0f} s, f32 {rec[name]['sha256_f32'][:16]}", flush=True)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
