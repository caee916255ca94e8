#!/usr/bin/env python3
"""A/B the render-kernel variants in ONE process, interleaved rounds (guide §5.4 rule 24).

Every variant must produce bit-identical frames; prints per-variant median/min kernel ms.
    python scripts/ab_variants.py [--config c3] [--rounds 5] [--variants exact:cull,exact:cull:transpose_max=0,...]
A variant is kind:traversal[:options][:s0]: kind exact|fast|scalar, traversal cull|brute,
options in rt_options_parse syntax with ';' between fields (each variant gets its own scene
with them, over the process default), s0: no segment counters. --stats: the instrumented kernel.
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import raytracinginoneweekend_amd as rt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--camera", default="reference")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--depth", type=int, default=0, help="override the config's max depth")
ap.add_argument("--spp", type=int, default=0, help="override the config's samples per pixel")
ap.add_argument("--variants", default="exact:cull,exact:brute,fast:cull,fast:brute")
ap.add_argument("--stats", action="store_true", help="the instrumented kernel (counters and per-wave timeline)")
ap.add_argument("--timeline-out", default="", help="with --stats: dump raw per-wave records to <prefix>.<variant>.json")
a = ap.parse_args()
scene, W, H, spp, depth = CONFIGS[a.config]
depth = a.depth or depth
spp = a.spp or spp
arrays = rt.huge_scene_arrays(1234) if scene == "huge" else rt.simple_scene_arrays()
cam = rt.Camera.default(W, H, rt.CORRECTED if a.camera == "corrected" else rt.REFERENCE)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
seg = torch.zeros(3, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
variants = [(v.split(":")[0], v.split(":")[1], v.split(":")[2:]) for v in a.variants.split(",")]
times = {":".join([k, t] + x): [] for k, t, x in variants}
scenes = {}
for kind, trav, extra in variants:
    o = rt.parse_options(";".join(x for x in extra if x != "s0"), rt.default_options())
    if a.stats:
        o = rt.options(o, stats=True)
    scenes[":".join([kind, trav] + extra)] = rt.DeviceScene(arrays, options=o)
ref = None
segs = {}
for r in range(a.rounds + 1):
    for kind, trav, extra in variants:
        ds = scenes[":".join([kind, trav] + extra)]
        p = rt.make_params(W, H, spp, depth, 1234, scalar_scene=kind == "scalar", fast_math=kind == "fast",
                           brute_force=trav == "brute")
        seg.zero_()
        count = not any(x == "s0" for x in extra)  # "s0": no segment counters (no end-of-kernel atomics)
        ds.render(cam, p, out.data_ptr(), stream, seg.data_ptr() if count else None)
        torch.cuda.synchronize()
        ms = ds.kernel_times(1)[0]
        name = ":".join([kind, trav] + extra)
        if r == 0:  # warm-up round: check bits
            img = out.cpu()
            if ref is None:
                ref = img
            same = torch.equal(img.view(torch.int32), ref.view(torch.int32))
            segs[name] = [int(x) for x in seg.tolist()]
            d = (img - ref).abs()
            px = d.amax(dim=-1)
            print(f"{name}: identical={same} segments={segs[name]} max|d|={d.max().item():.3g} "
                  f"mean|d|={d.mean().item():.3g} px<=1e-4: {(px <= 1e-4).float().mean().item()*100:.3f}% "
                  f"px<=1e-3: {(px <= 1e-3).float().mean().item()*100:.3f}%", flush=True)
            if a.stats:
                cnt = ds.debug_counters()
                print(f"{name}: counters {cnt}", flush=True)
                tl = [r for r in ds.debug_timeline() if r[1] >= r[0] > 0]
                if tl:  # wave concurrency over the launch: how much of it is drain
                    t0 = cnt["launch_start"] or min(r[0] for r in tl)
                    T = max(r[1] for r in tl) - t0

                    def qs(vals, scale=1.0, nd=3):
                        v = sorted(vals)
                        return {f"p{int(f * 100)}": round(v[min(len(v) - 1, int(f * len(v)))] / scale, nd)
                                for f in (0.0, 0.01, 0.1, 0.5, 0.9, 0.99, 1.0)}
                    busy = sum(r[1] - t0 for r in tl) / (len(tl) * T)
                    print(f"{name}: waves={len(tl)} launch={T / 1e5:.3f}ms mean wave occupancy {busy:.3f}\n"
                          f"  dry   (frac) {qs([r[0] - t0 for r in tl], T)}\n"
                          f"  exit  (frac) {qs([r[1] - t0 for r in tl], T)}\n"
                          f"  drain (frac) {qs([r[1] - r[0] for r in tl], T)}\n"
                          f"  iterations   {qs([r[2] for r in tl], 1, 0)}\n"
                          f"  iters after dry {qs([r[5] for r in tl], 1, 0)}\n"
                          f"  refills      {qs([r[4] for r in tl], 1, 0)}", flush=True)
                    dump = a.timeline_out
                    if dump:  # raw per-wave records for offline analysis
                        with open(f"{dump}.{name.replace(':', '_')}.json", "w") as fh:
                            json.dump(ds.debug_timeline(), fh)
                    late = sorted(tl, key=lambda r: -r[1])[:5]
                    print("  latest waves (dry, exit frac, iters, cu, refills, iters after dry):",
                          [(round((r[0] - t0) / T, 3), round((r[1] - t0) / T, 3), r[2], r[3], r[4], r[5]) for r in late],
                          flush=True)
        else:
            times[name].append(ms)
res = {}
for name, t in times.items():
    prim = W * H * spp
    res[name] = {"median_ms": round(statistics.median(t), 3), "min_ms": round(min(t), 3),
                 "mrays": round(prim / statistics.median(t) / 1e3, 1),
                 "exec_tflops": round((segs[name][1] * 20 + segs[name][2] * 19) / statistics.median(t) / 1e9, 2),
                 "tests_per_seg": round(segs[name][1] / max(1, segs[name][0]), 1),
                 "boxes_per_seg": round(segs[name][2] / max(1, segs[name][0]), 1)}
    print(name, json.dumps(res[name]), flush=True)
