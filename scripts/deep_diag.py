#!/usr/bin/env python3
"""The deep launch of a lone config-3 frame under the instrumented kernel (options stats=1,
stats_deep_only=1): block events per iteration, cycle shares per loop region, and the per-wave
timeline (when each wave found the queues dry, exited, its iterations) — for each --options.
    python scripts/deep_diag.py [--options "no_trap_loop=1" ...]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import raytracinginoneweekend_amd as rt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--options", nargs="*", default=[""])
ap.add_argument("--depth", type=int, default=0, help="override the config's max depth")
ap.add_argument("--spp", type=int, default=0, help="override the config's samples per pixel")
a = ap.parse_args()
scene, W, H, spp, depth = CONFIGS[a.config]
depth = a.depth or depth
spp = a.spp or spp
arrays = rt.huge_scene_arrays(1234) if scene == "huge" else rt.simple_scene_arrays()
cam = rt.Camera.default(W, H)
p = rt.make_params(W, H, spp, depth, 1234)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
def _qs(v):
    return [round(v[min(len(v) - 1, int(f * len(v)))], 3) if v else None for f in (0.0, 0.1, 0.5, 0.9, 1.0)]


for text in a.options:
    o = rt.parse_options(text, rt.options(rt.default_options(), stats=True, stats_deep_only=True))
    ds = rt.DeviceScene(arrays, options=o)
    for _ in range(2):  # the second lone frame is reported
        torch.cuda.synchronize()
        ds.debug_counters(reset=True)
        ds.debug_events(reset=True)
        ds.render(cam, p, out.data_ptr(), stream)
        torch.cuda.synchronize()
    c, ev = ds.debug_counters(reset=True), ds.debug_events(reset=True)
    tl = [r for r in ds.debug_timeline() if r[1] >= r[0] > 0]
    t0 = c["launch_start"] or (min(r[0] for r in tl) if tl else 0)
    cyc = sum(c[k] for k in ("cyc_refill", "cyc_start", "cyc_hit", "cyc_shade", "cyc_fold"))
    busy = [r for r in tl if r[2] > 0]
    ends = sorted(r[1] - t0 for r in busy)
    q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))] / 100.0 if v else None  # noqa: E731  (100 MHz ticks -> us)
    res = {"options": text, "lone_frame_ms": ds.kernel_times(1)[0], "waves": len(tl), "busy_waves": len(busy),
           "wave_iters": c["wave_iters"], "refills": c["wave_refills"],
           "cycle_share": {k: round(c[k] / max(1, cyc), 3) for k in ("cyc_refill", "cyc_start", "cyc_hit", "cyc_shade", "cyc_fold")},
           "cycles_per_wave_iter": round(cyc / max(1, c["wave_iters"]), 1),
           # shader clock seen by the waves: their s_memtime cycles over their s_memrealtime life
           # (every wave of the resident grid starts at the launch's start)
           "clock_ghz_busy_waves": {f"p{int(f * 100)}": v for f, v in zip(
               (0.0, 0.1, 0.5, 0.9, 1.0), _qs(sorted(r[7] / max(1, r[1] - r[6]) * 0.1 for r in busy)))},
           "us_per_busy_iter": {f"p{int(f * 100)}": v for f, v in zip(
               (0.0, 0.1, 0.5, 0.9, 1.0), _qs(sorted((r[1] - r[6]) / 100.0 / max(1, r[2]) for r in busy)))},
           "busy_wave_start_us": {f"p{int(f * 100)}": q(sorted(r[6] - t0 for r in busy), f) for f in (0.0, 0.5, 1.0)},
           "events": {k: int(v) for k, v in ev.items() if v},
           "busy_wave_exit_us": {f"p{int(f * 100)}": q(ends, f) for f in (0.0, 0.1, 0.5, 0.9, 0.99, 1.0)},
           "busy_wave_dry_us": {f"p{int(f * 100)}": q(sorted(r[0] - t0 for r in busy), f) for f in (0.0, 0.1, 0.5, 0.9, 1.0)},
           "idle_wave_exit_us": {f"p{int(f * 100)}": q(sorted(r[1] - t0 for r in tl if r[2] == 0), f)
                                 for f in (0.0, 0.1, 0.5, 0.9, 1.0)},
           "iters_per_busy_wave": {f"p{int(f * 100)}": (sorted(r[2] for r in busy)[min(len(busy) - 1, int(f * len(busy)))] if busy else None)
                                   for f in (0.0, 0.5, 0.9, 1.0)}}
    res["paths_dealt"] = c.get("items_dealt", 0)
    res["deep_launch"] = ds.usage().get("deep_launch")
    # per busy wave: life (us), iterations, iterations in which it walked; the slowest and fastest tenth
    life = sorted(((r[1] - r[6]) / 100.0, r[2], r[5]) for r in busy)
    if life:
        k = max(1, len(life) // 10)
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        res["fastest_tenth"] = {"life_us": med([x[0] for x in life[:k]]), "iters": med([x[1] for x in life[:k]]),
                                "walk_iters": med([x[2] for x in life[:k]])}
        res["slowest_tenth"] = {"life_us": med([x[0] for x in life[-k:]]), "iters": med([x[1] for x in life[-k:]]),
                                "walk_iters": med([x[2] for x in life[-k:]])}
        # record word 0 of a deep launch: walks with a hint-less walking lane << 32 | walks
        nh = {id(r): (r[0] >> 32) for r in busy}
        res["slowest_tenth"]["walks_with_hintless_lane"] = med([nh[id(r)] for r in sorted(busy, key=lambda r: r[1] - r[6])[-k:]])
        res["fastest_tenth"]["walks_with_hintless_lane"] = med([nh[id(r)] for r in sorted(busy, key=lambda r: r[1] - r[6])[:k]])
        res["walk_iters_per_busy_wave"] = {f"p{int(f * 100)}": sorted(x[2] for x in life)[min(len(life) - 1, int(f * len(life)))]
                                           for f in (0.0, 0.5, 0.9, 1.0)}
    res["segments"] = c["segments"]
    its = sorted(r[2] for r in busy)
    hist = {}
    for v in its:
        hist[v // 8 * 8] = hist.get(v // 8 * 8, 0) + 1
    res["iters_hist_by8"] = dict(sorted(hist.items()))
    res["refills_per_busy_wave"] = {f"p{int(f * 100)}": (sorted(r[4] for r in busy)[min(len(busy) - 1, int(f * len(busy)))] if busy else None)
                                    for f in (0.0, 0.5, 0.9, 1.0)}
    print(json.dumps(res), flush=True)
    ds.close()
