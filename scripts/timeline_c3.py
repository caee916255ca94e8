#!/usr/bin/env python3
"""Where a lone frame's render launch spends its time (rt_options stats=1 build of the render
kernel): per-wave times at which the wave found every item queue dry and at which it exited,
relative to the earliest wave start, plus the same frame's uninstrumented single-launch time.
    python scripts/timeline_c3.py [--config c3] [--camera reference] [--rehearse-world N]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracinginoneweekend_amd as rt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--camera", default="reference")
ap.add_argument("--rehearse-world", type=int, default=1, help="render rank 0's rows of an N-way split")
a = ap.parse_args()
scene, W, H, spp, depth = CONFIGS[a.config]
arrays = rt.huge_scene_arrays(1234) if scene == "huge" else rt.simple_scene_arrays()
cam = rt.Camera.default(W, H, rt.CORRECTED if a.camera == "corrected" else rt.REFERENCE)
ds = rt.DeviceScene(arrays, options=rt.options(rt.default_options(), stats=True))
N = a.rehearse_world
rows = (H + N - 1) // N
out = torch.empty((rows, W, 3), dtype=torch.float32, device="cuda")
p = rt.make_params(W, H, spp, depth, 1234, row_offset=0, row_stride=N)
stream = torch.cuda.current_stream().cuda_stream
for _ in range(2):
    ds.render(cam, p, out.data_ptr(), stream)
    torch.cuda.synchronize()
ds.debug_counters(reset=True)
ds.render(cam, p, out.data_ptr(), stream)
torch.cuda.synchronize()
c = ds.debug_counters(reset=True)
tl = ds.debug_timeline()
dry = np.array([w[0] for w in tl], dtype=np.float64)
ext = np.array([w[1] for w in tl], dtype=np.float64)
iters = np.array([w[2] for w in tl], dtype=np.float64)
after = np.array([w[5] for w in tl], dtype=np.float64)
start = float(c["launch_start"]) or min(dry.min(), ext.min())  # 100 MHz ticks
rec = {"config": a.config, "camera": a.camera, "rehearse_world": N, "waves": len(tl)}
span = ext.max() - start
q = lambda x, f: round(float(np.quantile((x - start) / span, f)), 3)  # noqa: E731
rec["launch_us"] = round(span * 0.01, 1)
rec["dry_frac_of_launch"] = {f"q{int(f*100)}": q(dry, f) for f in (0.01, 0.1, 0.5, 0.9, 0.99)}
rec["exit_frac_of_launch"] = {f"q{int(f*100)}": q(ext, f) for f in (0.01, 0.1, 0.5, 0.9, 0.99, 1.0)}
rec["iters_per_wave"] = {"mean": round(float(iters.mean()), 1), "max": int(iters.max())}
rec["iters_after_dry"] = {"mean": round(float(after.mean()), 1), "q90": float(np.quantile(after, .9)),
                          "max": int(after.max())}
print(json.dumps(rec))
