#!/usr/bin/env python3
"""Timeline of a bench run from a rocprofv3 --kernel-trace CSV: per render dispatch its queue,
start (relative to the first render of the window), duration, the previous render's start
(period), how many renders ran beside it, and the lag of its accumulation behind it; plus the
share of the window with 0..k renders running and the gaps where none ran.

    python scripts/trace_timeline.py <run_kernel_trace.csv> [--last 26]
"""
import argparse
import csv
import sys

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last", type=int, default=26, help="renders at the end of the run to show")
a = ap.parse_args()

rows = list(csv.DictReader(open(a.csv)))
ev = []
for r in rows:
    name = r["Kernel_Name"]
    kind = "render" if "render_kernel" in name else "accum" if "accumulate_kernel" in name else \
        "epi" if "epilogue" in name else "other"
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, int(r["Queue_Id"]), name[:60],
               int(r["Grid_Size_X"])))
ev.sort()
renders = [e for e in ev if e[2] == "render"][-a.last:]
if not renders:
    sys.exit("no render_kernel dispatches")
t0 = renders[0][0]
t_end = max(e[1] for e in renders)
accs = [e for e in ev if e[2] == "accum" and e[0] >= t0]
print(f"{'#':>3} {'q':>2} {'start_us':>9} {'dur_us':>8} {'d_start':>8} {'grid':>7} {'beside':>6}")
prev = None
for i, (s, e, _, q, _, g) in enumerate(renders):
    beside = sum(1 for (s2, e2, *_ ) in renders if s2 < e and e2 > s) - 1
    print(f"{i:3d} {q:2d} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {((s - prev) / 1e3 if prev else 0):8.1f} "
          f"{g // 256:7d} {beside:6d}")
    prev = s
print(f"accumulations in window: {len(accs)}, mean {sum(e - s for s, e, *_ in accs) / max(len(accs), 1) / 1e3:.1f} us")
# coverage: time with k renders in flight
pts = sorted([(s, 1) for s, *_ in renders] + [(e, -1) for _, e, *_ in renders])
cov, k, last = {}, 0, pts[0][0]
for t, dk in pts:
    cov[k] = cov.get(k, 0) + (t - last)
    k += dk
    last = t
span = t_end - t0
print("window %.1f us; share with k renders running: " % (span / 1e3)
      + ", ".join(f"{k}: {v / span:.3f}" for k, v in sorted(cov.items())))
# busy union of everything (renders + others) in the window
allk = sorted((s, e) for s, e, *_ in ev if e > t0 and s < t_end)
busy, cs, ce = 0, None, None
for s, e in allk:
    s, e = max(s, t0), min(e, t_end)
    if cs is None or s > ce:
        if cs is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"any kernel running: {busy / span:.3f} of the window")
