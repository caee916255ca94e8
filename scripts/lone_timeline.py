#!/usr/bin/env python3
"""Per-frame kernel timeline of lone frames from a rocprofv3 --kernel-trace CSV: for each frame
(a main render_kernel launch and what follows it) the main, deep and accumulation launches'
start offsets and durations in microseconds (main, deep, sky, acc).
    python scripts/lone_timeline.py <run_kernel_trace.csv> [...]
"""
import csv
import statistics
import sys

for path in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        short = ("deep" if "render_deep_kernel" in name else "main" if "render_kernel" in name
                 else "acc" if "accumulate_kernel" in name else "sky" if "sky_kernel" in name else None)
        if short is None:
            continue
        if short == "main":
            cur = {"t0": t0, "k": []}
            frames.append(cur)
        if cur is not None:
            cur["k"].append((short, (t0 - cur["t0"]) / 1e3, (t1 - t0) / 1e3, (t1 - cur["t0"]) / 1e3))
    print(path)
    spans = []
    for f in frames[1:]:
        spans.append(max(k[3] for k in f["k"]))
        print("  " + "  ".join(f"{n}@{s:.0f}+{d:.0f}" for n, s, d, e in f["k"]) + f"  end {spans[-1]:.0f} us")
    if spans:
        print(f"  median frame span {statistics.median(spans):.0f} us over {len(spans)} frames")
