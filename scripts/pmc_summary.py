#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv passes: per-kernel mean of each counter per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "render_kernel"
vals = defaultdict(list)
dur = []
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if filt not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    by = defaultdict(list)
    for (d, c), v in per.items():
        by[c].append(v)
    for c, v in by.items():
        vals[c].append(sum(v) / len(v))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for c in sorted(vals):
    print(f"{c:28s} {sum(vals[c])/len(vals[c]):.6g}")
if dur:
    print(f"{'duration_ms(mean)':28s} {sum(dur)/len(dur):.4f}  (n={len(dur)})")
