#!/usr/bin/env python3
"""Wave-level efficiency counters of the instrumented render kernel (rt_options stats=1) on a
bench config: live lanes per wave iteration, lane occupancy of the member-sphere blocks and of
the root work, cycles per loop region.   python scripts/stats_c3.py [--config c3]
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
ap.add_argument("--camera", default="reference")
a = ap.parse_args()
scene, W, H, spp, depth = CONFIGS[a.config]
arrays = rt.huge_scene_arrays(1234) if scene == "huge" else rt.simple_scene_arrays()
cam = rt.Camera.default(W, H, rt.CORRECTED if a.camera == "corrected" else rt.REFERENCE)
ds = rt.DeviceScene(arrays, options=rt.options(rt.default_options(), stats=True))
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
seg = torch.zeros(3, dtype=torch.int64, device="cuda")
p = rt.make_params(W, H, spp, depth, 1234)
stream = torch.cuda.current_stream().cuda_stream
ds.render(cam, p, out.data_ptr(), stream, seg.data_ptr())  # warm-up
torch.cuda.synchronize()
ds.debug_counters(reset=True)
ds.debug_events(reset=True)
seg.zero_()
ds.render(cam, p, out.data_ptr(), stream, seg.data_ptr())
torch.cuda.synchronize()
c = ds.debug_counters(reset=True)
ev = ds.debug_events(reset=True)
segments, sph, box = (int(x) for x in seg.cpu())
n_always = 1 if scene == "huge" else 0
member_tests = sph - n_always * segments
cyc = sum(c[k] for k in ("cyc_refill", "cyc_start", "cyc_hit", "cyc_shade", "cyc_fold"))
res = {
    "segments": segments,
    "wave_iters": c["wave_iters"],
    "live_lanes_per_iter": segments / max(1, c["wave_iters"]),
    "member_tests_lane": member_tests,
    "member_slots_wave": c["wave_member_blocks"] * 8 * 64,
    "member_lane_efficiency": member_tests / max(1, c["wave_member_blocks"] * 8 * 64),
    "blocks_lane_per_wave": c["lane_blocks"] / max(1, c["wave_blocks"]),
    "roots_lane_per_wave": c["lane_roots"] / max(1, c["wave_roots"]),
    "cycle_share": {k: round(c[k] / max(1, cyc), 3) for k in ("cyc_refill", "cyc_start", "cyc_hit", "cyc_shade", "cyc_fold")},
    "events_per_iter": {k: round(v / max(1, ev["iter"]), 4) for k, v in ev.items()},
    "raw": {k: int(v) for k, v in c.items()},
}
print(json.dumps(res, indent=1))
