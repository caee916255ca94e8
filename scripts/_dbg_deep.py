import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import raytracinginoneweekend_amd as rt
import oracle_binding as O
s, m = rt.huge_scene_arrays(1234)
W, H = 1280, 720
cam = O.camera_default(W, H, 1)
for brute in (True, False):
    p = rt.make_params(W, H, 2, 64, 1234, row_offset=300, row_stride=1, num_rows=1, brute_force=brute)
    want, seg = O.render_f32(s, m, cam, p)
    for dd in ("0", "2", "2", "3"):
        os.environ["RT_DEEP_DEPTH"] = dd
        got, st = rt.render_f32((s, m), p, cam)
        bad = np.argwhere((got.view(np.uint32) != want.view(np.uint32)).any(-1))
        print(f"brute={brute} deep={dd} segs {st.segments} vs {seg} bad px {len(bad)} first {bad[:6].tolist()}", flush=True)
