#!/usr/bin/env python3
"""Static instruction counts of one render_kernel instantiation per source line (VALU / SALU /
other), from a -gline-tables-only build of rt_kernel.hip: where the code of the hot loop sits.
U = VALU issue units by the gfx950 cost classes measured with scripts/ubench_int.hip (1: f32
add/sub/mul/fma, add/sub/and/or/xor/not/lshr u32, moves of VGPRs and literals; 2: every other
VALU op and any VALU op that reads an SGPR; 4: transcendental), G = VALU ops reading an SGPR.
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
FAST = {"v_fma_f32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_add_u32", "v_sub_u32",
        "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32", "v_lshrrev_b32", "v_mov_b32"}
TRANS = ("v_rcp_", "v_sqrt_", "v_exp_", "v_log_", "v_rsq_", "v_sin_", "v_cos_")
SREG = re.compile(r"^-?\|?s(\d+|\[)")


def valu_cost(line):
    parts = line.split(None, 1)
    op = re.sub(r"_e(32|64)$|_dpp$|_sdwa$", "", parts[0])
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    skip = 2 if op.startswith(("v_mad_u64", "v_mad_i64", "v_add_co", "v_sub_co", "v_addc", "v_subb")) else \
        (1 if op.startswith("v_cmp") else 1)
    sg = any(SREG.match(o) for o in ops[skip:])
    if op.startswith(TRANS):
        return 4, sg
    if op in FAST and not sg and "_dpp" not in parts[0]:
        return 1, sg
    return 2, sg
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
    if op.startswith("v_"):
        u, sg = valu_cost(line)
        cnt[cur]["U"] += u
        cnt[cur]["G"] += sg
text = open(os.path.join(src_dir, "rt_kernel.hip")).read().split("\n")
tot = collections.Counter()
for k in sorted(cnt, key=lambda k: (k or ("", 0))):
    c = cnt[k]
    tot.update(c)
    if sum(c.values()) < a.min:
        continue
    f, ln = k if k else ("?", 0)
    t = text[ln - 1].strip()[:72] if f == "rt_kernel.hip" and ln > 0 else ""
    print(f"{f}:{ln:<5d} V{c['V']:5d} U{c['U']:5d} G{c['G']:4d} S{c['S']:5d} M{c['M']:4d}  {t}")
print("total", dict(tot))
