#!/usr/bin/env python3
"""Host cost of issuing frames: N frames of config 3 (or a row share r/N) issued back to back
through DeviceScene.render; the host time of the issue loop alone vs the time to its last
frame's completion. If the two agree, the frame stream is bound by the host's issue, not the GPU.
    python scripts/host_probe.py --rows 0/8 --frames 40
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import raytracinginoneweekend_amd as rt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", default="")
ap.add_argument("--frames", type=int, default=40)
a = ap.parse_args()
scene, W, H, spp, depth = CONFIGS["c3"]
arrays = rt.huge_scene_arrays(1234)
cam = rt.Camera.default(W, H)
kw = {}
if a.rows:
    r, n = map(int, a.rows.split("/"))
    kw = dict(row_offset=r, row_stride=n, num_rows=(H - r + n - 1) // n)
p = rt.make_params(W, H, spp, depth, 1234, **kw)
outs = [torch.empty((rt.abi.rows_of(p), W, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
stream = torch.cuda.current_stream().cuda_stream
ds = rt.DeviceScene(arrays)
for i in range(10):
    ds.render(cam, p, outs[i % 2].data_ptr(), stream)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    per = []
    for i in range(a.frames):
        t = time.perf_counter()
        ds.render(cam, p, outs[i % 2].data_ptr(), stream)
        per.append(time.perf_counter() - t)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    per.sort()
    print({"rows": a.rows or "all", "issue_ms_per_frame": round((t1 - t0) / a.frames * 1e3, 4),
           "done_ms_per_frame": round((t2 - t0) / a.frames * 1e3, 4),
           "render_call_ms_p50": round(per[len(per) // 2] * 1e3, 4), "render_call_ms_p90": round(per[int(len(per) * 0.9)] * 1e3, 4)},
          flush=True)
ds.close()
