#!/usr/bin/env python3
"""TEST INFRASTRUCTURE (analysis only): where the deep paths of a config-3 frame come from.

Traces every sample of a frame on the CPU with the restatement (tests/tools/deep_sources.cpp,
which includes oracle/rt_oracle.cpp) and reports, for the samples that trace more than
`--split` segments (the deep paths): the kind of their primary hit, the segment
of their first dielectric hit, and how they spread over the frame's 8x8 tiles, split by the
tiles' classes (a tile whose primaries hit a dielectric sphere / hit anything / all reach the
sky). The result decides the dealing order of a lone pass.

    python tests/tools/deep_sources.py [--spp 16] [--threads 8] > profiles/r06/deep_sources.txt
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def build():
    out = os.path.join(REPO, "tests", "tools", "_build", "libdeep_sources.so")
    src = os.path.join(REPO, "tests", "tools", "deep_sources.cpp")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(out), exist_ok=True)
        subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-pthread",
                        "-shared", "-o", out, src], check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=1280)
    ap.add_argument("--h", type=int, default=720)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--depth", type=int, default=64)
    ap.add_argument("--split", type=int, default=8)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    import raytracinginoneweekend_amd as rt
    from raytracinginoneweekend_amd import _abi as abi
    import oracle_binding as O
    L = C.CDLL(build())
    L.deep_sources.restype = C.c_int
    W, H, spp = args.w, args.h, args.spp
    s, m = rt.huge_scene_arrays(1234)
    cam = O.camera_default(W, H, 0)
    p = rt.make_params(W, H, spp, args.depth, 1234)
    n = W * H * spp
    segs = np.zeros(n, np.uint32)
    prim = np.zeros(n, np.uint8)
    fdi = np.zeros(n, np.uint8)
    sa = abi.ptr(s, C.POINTER(abi.RtSphere))
    ma = abi.ptr(m, C.POINTER(abi.RtMaterial))
    rc = L.deep_sources(sa, len(s), ma, len(m), C.byref(cam), C.byref(p), args.threads,
                        segs.ctypes.data_as(C.c_void_p), prim.ctypes.data_as(C.c_void_p),
                        fdi.ctypes.data_as(C.c_void_p))
    assert rc == 0
    segs = segs.reshape(H, W, spp)
    prim = prim.reshape(H, W, spp)
    fdi = fdi.reshape(H, W, spp)
    deep = segs > args.split
    nd = int(deep.sum())
    print(f"frame {W}x{H} @{spp} spp, huge scene seed 1234, reference camera, depth {args.depth}")
    print(f"samples {n}, segments {int(segs.sum())} ({segs.sum() / n:.4f} per primary)")
    print(f"deep samples (> {args.split} segments): {nd} ({nd / n * 100:.4f}%), "
          f"reaching max depth: {int((segs >= args.depth).sum())}")
    names = ["sky", "lambert sphere", "metal", "dielectric", "ground"]
    print("primary hit of the deep samples:",
          ", ".join(f"{names[k]} {int((prim[deep] == k).sum())}" for k in range(5)))
    fd = fdi[deep]
    print("first dielectric hit of the deep samples: segment 1 %d, 2 %d, 3 %d, 4-8 %d, later %d, none %d" % (
        int((fd == 1).sum()), int((fd == 2).sum()), int((fd == 3).sum()), int(((fd >= 4) & (fd <= 8)).sum()),
        int((fd > 8).sum()), int((fd == 0).sum())))
    # 8x8 tiles: classes by the primary hits of all their samples
    th, tw = H // 8, W // 8
    t = lambda a: a[:th * 8, :tw * 8].reshape(th, 8, tw, 8, *a.shape[2:]).swapaxes(1, 2).reshape(th, tw, -1)  # noqa: E731
    tp, tdeep, tseg = t(prim), t(deep), t(segs)
    has_d = (tp == 3).any(-1)
    has_s = ((tp == 1) | (tp == 2)).any(-1)
    has_hit = (tp > 0).any(-1)
    cls = np.where(has_d, 0, np.where(has_s, 1, np.where(has_hit, 2, 3)))
    print(f"8x8 tiles: {th * tw}")
    for c, name in enumerate(["a primary hits a dielectric", "a primary hits another small sphere",
                              "primaries hit the ground only", "every primary reaches the sky"]):
        sel = cls == c
        print(f"  class {c} ({name}): {int(sel.sum())} tiles ({sel.mean() * 100:.1f}%), "
              f"segments {tseg[sel].sum() / segs.sum() * 100:.1f}% of the frame's, "
              f"deep samples {int(tdeep[sel].sum())} ({tdeep[sel].sum() / max(nd, 1) * 100:.1f}%)")
    per_tile = np.sort(tdeep.sum(-1).ravel())[::-1]
    cum = np.cumsum(per_tile) / max(nd, 1)
    for frac in (0.5, 0.8, 0.9, 0.99):
        k = int(np.searchsorted(cum, frac)) + 1
        print(f"  {frac * 100:.0f}% of the deep samples lie in the {k} tiles with most of them ({k / (th * tw) * 100:.1f}%)")


if __name__ == "__main__":
    main()
