#!/usr/bin/env python3
"""rocprofv3 --pmc passes (pmc_round.sh layout: <root>/p*/run_counter_collection.csv and
run_kernel_trace.csv) split into the main launches (render_kernel) and the deep launches of
split passes (render_deep_kernel; builds before it had one kernel for both, told apart here by
duration: the deep launch is the shorter one, below --split-ms).
    python scripts/pmc_dispatch.py <root> [--split-ms 1.8]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--split-ms", type=float, default=1.8)
ap.add_argument("--timed", action="store_true",
                help="only the timed instantiations (render_kernel<0, 7, false, false>, render_deep_kernel<0, false, false, 4|8>)")
a = ap.parse_args()


def wanted(name):
    if "render_kernel" not in name and "render_deep_kernel" not in name:
        return False
    return not a.timed or "<0, 7, false, false, false>" in name or "render_deep_kernel<0, false, false" in name

groups = {"main": defaultdict(list), "deep": defaultdict(list)}
for d in sorted(x for x in glob.glob(os.path.join(a.root, "p*")) if os.path.isdir(x)):
    dur, deep = {}, set()
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        if wanted(r["Kernel_Name"]):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            if "render_deep_kernel" in r["Kernel_Name"]:
                deep.add(r["Dispatch_Id"])
    per = defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if wanted(r["Kernel_Name"]):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    def kind(di):
        if deep:
            return "deep" if di in deep else "main"
        return "main" if dur[di] >= a.split_ms else "deep"
    for (di, c), v in per.items():
        if di in dur:
            groups[kind(di)][c].append(v)
    for di, t in dur.items():
        groups[kind(di)]["duration_ms"].append(t)
for g, vals in groups.items():
    n = len(vals.get("duration_ms", []))
    print(f"== {g} launches (n={n} dispatches over the passes)")
    for c in sorted(vals):
        v = vals[c]
        print(f"  {c:28s} {sum(v) / len(v):.6g}")
