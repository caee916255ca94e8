#!/usr/bin/env python3
"""Condense rocprofv3 --pmc passes of bench.py into the JSON bench.py reads for roofline.traffic.

    python scripts/pmc_json.py <pmc dir with p*/run_counter_collection.csv> <out.json> \
        [--kernel 'render_kernel<0, 7, false, false, false> + render_deep_kernel<0, false, false, 4|8>'] [--config c3]

Per frame (the kernel's dispatches of a frame summed, mean over frames and passes):
  hbm_bytes_per_frame  = 2 x FETCH_SIZE + WRITE_SIZE (KiB counters; FETCH_SIZE counts half of the
                         bytes of wide streaming reads on gfx950, MI355X_MICROARCH.md HBM section)
  valu_busy            = SQ_INSTS_VALU x 2 cycles / (SIMDs x GRBM_GUI_ACTIVE / 8)
                         (wave64 VALU issue = 2 cycles; GRBM_GUI_ACTIVE sums the 8 XCDs)
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("out")
ap.add_argument("--kernel", default="render_kernel<0, 7, false, false, false> + render_deep_kernel<0, false, false, 4|8> + sky_kernel",
                help="kernel names joined by ' + '; the first one's dispatches count the frames")
ap.add_argument("--config", default="c3")
ap.add_argument("--camera", default="reference")
ap.add_argument("--traversal", default="cull")
ap.add_argument("--simds", type=int, default=1024)  # 256 CUs x 4 SIMDs
a = ap.parse_args()
names = [k.strip() for k in a.kernel.split(" + ") if k.strip()]


def matches(k, kernel_name):
    """k in kernel_name; a last template argument 'a|b' matches either instantiation"""
    if "|" in k:
        pre, last = k.rsplit(", ", 1)
        return any(f"{pre}, {x}>" in kernel_name for x in last.rstrip(">").split("|"))
    return k in kernel_name


def which(kernel_name):
    return next((i for i, k in enumerate(names) if matches(k, kernel_name)), None)


# Per frame: every dispatch of the kernels in a pass summed and divided by the frames the pass's
# bench.py run issued to them (its JSON line's frames_issued, in <pass dir>.log; a frame is one
# pass issued alone or several ring passes beside other frames). Without that field: the first
# kernel's dispatches (one main launch per one-pass frame).
def pass_frames(path):
    top = os.path.relpath(path, a.root).split(os.sep)[0]
    try:
        with open(os.path.join(a.root, top + ".log")) as fh:
            line = [x for x in fh if x.startswith("{")][-1]
        return json.loads(line).get("frames_issued") or None
    except (OSError, IndexError, ValueError):
        return None


vals = defaultdict(list)
for f in sorted(glob.glob(os.path.join(a.root, "p*", "**", "run_counter_collection.csv"), recursive=True)):
    per = defaultdict(float)
    frames = set()
    for r in csv.DictReader(open(f)):
        i = which(r["Kernel_Name"])
        if i is None:
            continue
        if i == 0:
            frames.add(r["Dispatch_Id"])
        per[r["Counter_Name"]] += float(r["Counter_Value"])
    nf = pass_frames(f) or len(frames)
    for c, v in per.items():
        vals[c].append(v / nf)
dur = []
for f in sorted(glob.glob(os.path.join(a.root, "p*", "**", "run_kernel_trace.csv"), recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if which(r["Kernel_Name"]) is not None]
    n = pass_frames(f) or sum(1 for r in rows if which(r["Kernel_Name"]) == 0)
    if n:
        dur.append(sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rows) / n)
m = {c: sum(v) / len(v) for c, v in vals.items()}
need = ["FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"]
missing = [c for c in need if c not in m]
if missing:
    raise SystemExit(f"missing counters {missing} for kernel {a.kernel!r} under {a.root}")
from bench import WORKLOAD, kernel_sha256, lib_sha256  # noqa: E402

if kernel_sha256() is None:
    raise SystemExit("a timed kernel's symbol (bench.TIMED_KERNEL) is missing from the loaded library")
t = sum(dur) / len(dur)
cycles = m["GRBM_GUI_ACTIVE"] / 8.0
rec = {
    "kernel": " + ".join(names),
    # the build these counters describe: bench.py uses them only for the same library
    "kernel_sha256": kernel_sha256(),
    "lib_sha256": lib_sha256(),
    "config": {"workload": WORKLOAD[a.config], "camera": a.camera, "traversal": a.traversal, "n_gpus": 1},
    # per frame: the kernel's dispatches of one frame (durations summed: a span of overlapping
    # launches when frames are in flight)
    "kernel_ms_per_frame": round(t * 1e3, 4),
    "clock_ghz": round(cycles / t / 1e9, 3),
    "hbm_bytes_per_frame": int(2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024),
    "fetch_bytes_corrected": int(2 * m["FETCH_SIZE"] * 1024),
    "write_bytes": int(m["WRITE_SIZE"] * 1024),
    "valu_insts": m["SQ_INSTS_VALU"],
    "valu_busy": round(m["SQ_INSTS_VALU"] * 2.0 / (a.simds * cycles), 4),
    "valu_lane_ops_per_s": m["SQ_INSTS_VALU"] * 64 / t,
    "counters": {c: m[c] for c in sorted(m)},
}
with open(a.out, "w") as f:
    json.dump(rec, f, indent=1)
print(json.dumps({k: v for k, v in rec.items() if k != "counters"}))
