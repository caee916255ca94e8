#!/usr/bin/env python3
"""Static instruction counts of one render_kernel instantiation per source line (VALU / SALU /
other), from a -gline-tables-only build of rt_kernel.hip: where the code of the hot loop sits.
    python scripts/asm_lines.py [--kernel _ZN2rt13render_kernelILi0ELi7ELb0EEEvNS_7KParamsE] [--min 6]
"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default="_ZN2rt13render_kernelILi0ELi7ELb0EEEvNS_7KParamsE")
ap.add_argument("--min", type=int, default=6)
ap.add_argument("--flags", default="")
a = ap.parse_args()
src_dir = os.path.join(REPO, "raytracinginoneweekend_amd", "csrc")
tmp = tempfile.mkdtemp()
subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fno-slp-vectorize", "--offload-arch=gfx950",
                "-ffp-contract=off", "-fno-fast-math", "-gline-tables-only", "-S", "--cuda-device-only",
                *a.flags.split(), os.path.join(src_dir, "rt_kernel.hip"), "-o", os.path.join(tmp, "k.s")], check=True)
s = open(os.path.join(tmp, "k.s")).read()
files = {m.group(1): m.group(3) or m.group(2) for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)}
i = s.index(a.kernel + ":")
j = s.index(".Lfunc_end", i)
cur = None
cnt = collections.defaultdict(collections.Counter)
for line in s[i:j].split("\n"):
    line = line.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", line)
    if m:
        cur = (os.path.basename(files.get(m.group(1), "?")), int(m.group(2)))
        continue
    if not line or line.startswith((".", ";", "//")) or line.endswith(":"):
        continue
    op = line.split()[0]
    cnt[cur]["V" if op.startswith("v_") else "S" if op.startswith("s_") else "M"] += 1
text = open(os.path.join(src_dir, "rt_kernel.hip")).read().split("\n")
tot = collections.Counter()
for k in sorted(cnt, key=lambda k: (k or ("", 0))):
    c = cnt[k]
    tot.update(c)
    if sum(c.values()) < a.min:
        continue
    f, ln = k if k else ("?", 0)
    t = text[ln - 1].strip()[:72] if f == "rt_kernel.hip" and ln > 0 else ""
    print(f"{f}:{ln:<5d} V{c['V']:5d} S{c['S']:5d} M{c['M']:4d}  {t}")
print("total", dict(tot))
