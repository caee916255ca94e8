#!/usr/bin/env python3
"""Config 4 (3840x2160 @256 spp, 13 passes) rendered under option variants and compared with the
reference's whole-frame digests (tests/golden/fullframe.json): rows that differ per variant.
    python scripts/c4_check.py "opt=v;opt=v" ...
"""
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import golden_io as G  # noqa: E402
import raytracinginoneweekend_amd as rt  # noqa: E402

ref = json.load(open(os.path.join(REPO, "tests", "golden", "fullframe.json")))["c4"]
s, m = G.scene("huge")
for text in sys.argv[1:] or [""]:
    rt.set_default_options(rt.parse_options(text, rt.options()))
    img, st = rt.render_f32((s, m), rt.make_params(3840, 2160, 256, 64, 1234, full_frame=True))
    bad = [y for y in range(2160) if hashlib.sha256(np.ascontiguousarray(img[y]).tobytes()).hexdigest()[:16]
           != ref["row_sha256_16"][y]]
    print(json.dumps({"options": text, "rows_differing": len(bad), "first": bad[:6], "last": bad[-3:],
                      "segments": st.segments}), flush=True)
