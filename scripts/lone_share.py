#!/usr/bin/env python3
"""Lone frames of config 3 (or one row share r/N of it), each issued alone and waited for: the
workload whose kernel timeline scripts/lone_timeline.py reads from a rocprofv3 --kernel-trace
CSV (the 8-way share's lone latency).
    rocprofv3 --kernel-trace --output-format csv -d out -o run -- python3 scripts/lone_share.py --rows 0/8
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import raytracinginoneweekend_amd as rt  # noqa: E402
from bench import CONFIGS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--rows", default="", help="row share r/N (e.g. 0/8)")
ap.add_argument("--frames", type=int, default=8)
ap.add_argument("--options", default="")
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
ds = rt.DeviceScene(arrays, options=rt.parse_options(a.options, rt.default_options()) if a.options else None)
ms = []
for _ in range(a.frames):
    torch.cuda.synchronize()
    ds.render(cam, p, out.data_ptr(), stream)
    torch.cuda.synchronize()
    ms.append(round(ds.kernel_times(1)[0], 3))
print({"rows": a.rows or "all", "frame_ms": ms, "usage": {k: v for k, v in ds.usage().items() if k in
       ("split_passes", "lead_tiles", "sky_tiles", "deep_launch")}}, flush=True)
ds.close()
