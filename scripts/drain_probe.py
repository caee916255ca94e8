#!/usr/bin/env python3
"""The main launch of a lone config-3 frame under the instrumented kernel (options stats=1): when
the waves found every queue dry (the last items dealt), when they exited, and how many iterations
they ran after the queues ran dry (the drain), for each --options. The
instrumented kernel runs at lower occupancy than the product: its times show the drain's shape,
not the product's durations.
    python scripts/drain_probe.py --options "" "natural_order=1,lone_split=1" ...
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
ap.add_argument("--rows", default="", help="row share r/N (e.g. 0/8)")
a = ap.parse_args()
scene, W, H, spp, depth = CONFIGS[a.config]
arrays = rt.huge_scene_arrays(1234) if scene == "huge" else rt.simple_scene_arrays()
cam = rt.Camera.default(W, H)
kw = {}
if a.rows:
    r, n = map(int, a.rows.split("/"))
    kw = dict(row_offset=r, row_stride=n, num_rows=(H - r + n - 1) // n)
p = rt.make_params(W, H, spp, depth, 1234, **kw)
out = torch.empty((rt.abi.rows_of(p), W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream


def qs(v, fs=(0.0, 0.1, 0.5, 0.9, 0.99, 1.0)):
    v = sorted(v)
    return {f"p{int(f * 100)}": (round(v[min(len(v) - 1, int(f * len(v)))], 1) if v else None) for f in fs}


for text in a.options:
    o = rt.parse_options(text, rt.options(rt.default_options(), stats=True))
    ds = rt.DeviceScene(arrays, options=o)
    for _ in range(2):  # the second lone frame is reported
        torch.cuda.synchronize()
        ds.debug_counters(reset=True)
        ds.debug_events(reset=True)
        ds.render(cam, p, out.data_ptr(), stream)
        torch.cuda.synchronize()
    c = ds.debug_counters(reset=True)
    u = ds.usage()
    tl = [r for r in ds.debug_timeline() if r[1] >= r[0] > 0]
    t0 = c["launch_start"] or (min(r[6] for r in tl) if tl else 0)
    us = lambda t: (t - t0) / 100.0  # noqa: E731  (100 MHz ticks)
    busy = [r for r in tl if r[2] > 0]
    res = {"options": text, "frame_ms": round(ds.kernel_times(1)[0], 3), "waves": len(tl),
           "lead_tiles": u["lead_tiles"], "sky_tiles": u["sky_tiles"], "split_passes": u["split_passes"],
           "dry_us": qs([us(r[0]) for r in busy]), "exit_us": qs([us(r[1]) for r in busy]),
           "iters_after_dry": qs([r[5] for r in busy]), "iters": qs([r[2] for r in busy]),
           "us_per_iter": qs([(r[1] - r[6]) / 100.0 / max(1, r[2]) for r in busy])}
    print(json.dumps(res), flush=True)
    ds.close()
