#!/usr/bin/env python3
"""Benchmark: Mrays/s + frame wall-clock on the huge random-sphere scene, 1280x720 @128spp
(BASELINE.json config 3), on 1..8 MI355X GPUs.

One step = one full frame: every rank renders its interleaved rows (y = rank + i*N) with
the HIP megakernel into HBM, the per-rank tiles are gathered to rank 0 over RCCL and
de-interleaved into the frame. Inputs (scene, camera) are resident in HBM before timing.
value = W*H*spp primary rays per frame * steps / max-over-ranks time (whole job).

Consecutive frames are in flight together (rt_render_device runs each render kernel on an
internal stream with its own workspace; results still land in caller-stream order),
so ms_per_step is the steady-state frame time; frame_latency_ms is one frame alone, start to
finish (render + accumulate + gather), timed synchronously after the timed loop.

    python bench.py [--gpus N --steps K --warmup W]     (N > 1: starts N ranks itself)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

parity: rank 0 hashes the last timed frame and compares it with the reference's own whole-frame
digest (tests/golden/fullframe.json, made from the reference's CPU path by
tests/golden/make_fullframe.py): "matches_reference" is true only if every bit agrees.

The cpu_baseline leg (rank 0, N=1) times the REFERENCE's own CPU path (oracle/_ref, built
from /root/reference) on a bounded row subset of the same workload, on this host's cores, with
a single-thread figure and the optimized CPU restatement beside it.

roofline: executed sphere + box test FLOP per frame over the frame period (ms_per_step) against
the f32 vector peak; traffic and VALU issue come from a rocprofv3 --pmc summary of the SAME
build of the timed kernel (profiles/pmc_render_c3.json, stamped with the sha256 of that kernel's
machine code and descriptor, kernel_sha256; dropped otherwise).
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_FP32_TFLOPS = 157.3   # MI355X f32 vector peak (MI355X_MICROARCH.md, chip-level table)
FLOP_PER_TEST = 20         # one ray-sphere test, SURVEY.md §8(d): 17 to the discriminant + 3 root
FLOP_PER_BOX = 19          # one padded cluster-AABB slab test
CONFIGS = {
    # name: (scene, W, H, spp, depth)
    "c3": ("huge", 1280, 720, 128, 64),
    "c2": ("simple", 1280, 720, 64, 50),
    "c4": ("huge", 3840, 2160, 256, 64),
    "c5": ("huge", 1280, 720, 1024, 64),
    "c1": ("simple", 200, 100, 1, 64),
    # the reference's CUDA variant (cuda_impl.cu): its scene, camera, 48 spp, 32 bounces
    "cuda": ("cuda", 1280, 720, 48, 32),
}
WORKLOAD = {
    "c3": "huge-scene 1280x720x128spp (BASELINE config 3)",
    "c2": "simple-scene 1280x720x64spp depth 50 (config 2)",
    "c4": "huge-scene 3840x2160x256spp (config 4)",
    "c5": "huge-scene 1280x720x1024spp (config 5)",
    "c1": "simple-scene 200x100x1spp (config 1)",
    "cuda": "cuda_impl preset: its 5-sphere scene 1280x720x48spp depth 32 (RT_FLAG_CUDA_COMPAT)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--camera", default="reference", choices=["reference", "corrected"])
    ap.add_argument("--variant", default="exact", choices=["exact", "fast", "scalar", "wavefront"],
                    help="exact: bit-exact kernel; fast: FMA kernel within the stated tolerance; "
                         "scalar: brute-force scalar-cache A/B; wavefront: per-segment launches with HBM ray queues "
                         "(A/B, bit-exact)")
    ap.add_argument("--traversal", default="cull", choices=["cull", "brute"],
                    help="cull: exact cluster culling (same bits); brute: every sphere, as the reference")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip dropin_first_ms / dropin_repeat_ms")
    ap.add_argument("--cpu-rows", type=int, default=240, help="rows in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every core this job may use (cpu_info)")
    ap.add_argument("--rehearse-world", type=int, default=0,
                    help="diagnostic, 1 GPU: render only rank 0's rows of an N-way split (no gather) to "
                         "estimate one rank's frame time at N GPUs; not a bench line")
    ap.add_argument("--rehearse-rank", type=int, default=0,
                    help="with --rehearse-world N: which rank's rows (default 0)")
    ap.add_argument("--rehearse-blocks", action="store_true",
                    help="with --rehearse-world N: the rank's rows as one contiguous block (H/N rows) instead of "
                         "every N-th row (A/B of the partition)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process, set before HIP starts (0: leave the environment, "
                         "HIP's default 4): the library runs one render stream fewer than this, 2..7 "
                         "(rt_host.cpp pipeline_env); the line records both values")
    ap.add_argument("--output", default="f32", choices=["f32", "rgb8"],
                    help="f32: the linear frame (12 B/pixel gathered); rgb8: gamma/u8 epilogue on every rank "
                         "before the gather (3 B/pixel), the reference's output format")
    ap.add_argument("--digest", action="store_true",
                    help="kept for old scripts: every line now carries parity.frame_sha256 (the last timed frame's "
                         "sha256 on rank 0) and its comparison with the reference's digest")
    ap.add_argument("--corrected-steps", type=int, default=5,
                    help="frames of the same workload with the corrected camera, reported as corrected_camera "
                         "(0: skip)")
    ap.add_argument("--rehearse-gather", action="store_true",
                    help="with --rehearse-world N: stand in for rank 0's gather with its device work on the "
                         "caller stream (the N-1 peer tiles copied into the gather buffer, then the "
                         "de-interleave copy), to see whether that work waits for CU slots")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_render_c3.json"),
                    help="PMC summary of this kernel (scripts/pmc_round.sh) for roofline.traffic / VALU busy")
    ap.add_argument("--options", default="",
                    help="rt_options for the scene, rt_options_parse syntax (e.g. 'max_workspace_bytes=4294967296,"
                         "render_streams=4'): over the library defaults and RT_OPTIONS; recorded in config.options")
    ap.add_argument("--launch-check", action="store_true",
                    help="launcher self-test (CPU): every rank joins a gloo group, prints its rank/world and "
                         "exits before any GPU call")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`bench.py --gpus N` started as ONE process: run N ranks under torch.distributed.run (one
    process per GPU, rendezvous on 127.0.0.1) and return its exit code. Called before this
    process touches the GPU (it never initialises HIP), so the ranks start clean."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the host driver's only mode)
    env.setdefault("OMP_NUM_THREADS", env.get("OMP_NUM_THREADS", "16"))
    return subprocess.call(cmd, env=env)


def env_int(name, default):
    """An integer from the environment, empty meaning the default (as rt_host.cpp reads it)."""
    v = os.environ.get(name, "")
    try:
        return int(v) if v.strip() else default
    except ValueError:
        return default


def reference_digest(config, W, H):
    """The reference's whole-frame digests for this config (tests/golden/fullframe.json, made by
    tests/golden/make_fullframe.py from the reference's own CPU path), or None."""
    try:
        with open(os.path.join(REPO, "tests", "golden", "fullframe.json")) as f:
            rec = json.load(f).get(config)
    except (OSError, ValueError):
        return None
    return rec if rec and rec["width"] == W and rec["height"] == H else None


def parity_record(frame_np, config, W, H, row_offset, row_stride, seed, camera, variant, output):
    """Compare the last timed frame (rank 0) with the reference's digests: the whole frame's
    sha256, or for a row share (rehearsal) the 64-bit row digests of the rows it rendered."""
    import hashlib
    rows = frame_np.shape[0]
    rec = {"frame_sha256": hashlib.sha256(frame_np.tobytes()).hexdigest()}
    ref = reference_digest(config, W, H)
    if output != "f32":
        rec.update(matches_reference=None, note="u8 output: the device epilogue is within 1 LSB of glibc powf, "
                                                "not bitwise; the f32 frame is the parity object")
        return rec
    if ref is None or seed != ref["seed"] or camera != ref["camera"]:
        rec.update(matches_reference=None, note="no reference digest for this config/seed/camera")
        return rec
    if row_stride == 1 and rows == ref["height"]:
        rec["reference_sha256"] = ref["sha256_f32"]
        rec["matches_reference"] = rec["frame_sha256"] == ref["sha256_f32"]
    else:
        got = [hashlib.sha256(frame_np[i].tobytes()).hexdigest()[:16] for i in range(rows)]
        want = [ref["row_sha256_16"][row_offset + i * row_stride] for i in range(rows)]
        bad = [row_offset + i * row_stride for i in range(rows) if got[i] != want[i]]
        rec.update(rows_checked=rows, rows_differing=len(bad), matches_reference=not bad)
    if variant == "fast":
        rec["note"] = "fast variant: within the stated tolerance, not bitwise by design"
    rec["reference"] = "tests/golden/fullframe.json[%s] (oracle/_ref/ref_harness_pcg, the reference's CPU path)" % config
    return rec


def lib_sha256():
    """sha256 of the product library this process loads: PMC summaries are stamped with it."""
    import hashlib
    from raytracinginoneweekend_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


# the timed kernels: rt::render_kernel<0, 7, false, false, false> (main launch, single samples),
# rt::render_deep_kernel<0, false, false, 4 | 8> (the deep launch of a split pass: 4-wave groups
# beside other renders, 8-wave groups for a lone pass) and rt::sky_kernel (the tiles proven to send
# every primary ray to the sky)
TIMED_KERNEL = ("_ZN2rt13render_kernelILi0ELi7ELb0ELb0ELb0EEEvNS_7KParamsE",
                "_ZN2rt18render_deep_kernelILi0ELb0ELb0ELi4EEEvNS_7KParamsE",
                "_ZN2rt18render_deep_kernelILi0ELb0ELb0ELi8EEEvNS_7KParamsE",
                "_ZN2rt10sky_kernelENS_4KSkyE")
TIMED_KERNEL_NAMES = ("render_kernel<0, 7, false, false, false> + render_deep_kernel<0, false, false, 4|8> + "
                      "sky_kernel")


def hashlib_sha256(b):
    import hashlib
    return hashlib.sha256(b).hexdigest()


def _elf_sections(b):
    import struct
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    stro = hdrs[shstrndx][4]
    return {b[stro + h[0]:b.index(b"\0", stro + h[0])].decode(): h for h in hdrs}, hdrs


def kernel_sha256(symbol=TIMED_KERNEL):
    """sha256 of the machine code and kernel descriptors of one kernel (a symbol) or several (a
    tuple) in the gfx950 code objects of the loaded library (PMC summaries are stamped with it,
    so host-side or other-instantiation changes do not invalidate them); None if a symbol is
    not found."""
    if isinstance(symbol, (tuple, list)):
        parts = [kernel_sha256(x) for x in symbol]
        if None in parts:
            return None
        return hashlib_sha256("".join(parts).encode())
    import hashlib
    import struct
    from raytracinginoneweekend_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        so = f.read()
    secs, _ = _elf_sections(so)
    h = secs[".hip_fatbin"]
    fat = so[h[4]:h[4] + h[5]]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    digest, pos = hashlib.sha256(), fat.find(magic)
    found = False
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" not in triple:
                continue
            co = fat[pos + off:pos + off + size]
            cs, hdrs = _elf_sections(co)
            if ".symtab" not in cs:
                continue
            sym, stra = cs[".symtab"], cs[".strtab"][4]
            for i in range(sym[5] // 24):
                name_off, info, other, shndx, value, ssize = struct.unpack_from("<IBBHQQ", co, sym[4] + 24 * i)
                name = co[stra + name_off:co.index(b"\0", stra + name_off)].decode()
                if name in (symbol, symbol + ".kd") and ssize:
                    sh = hdrs[shndx]
                    start = sh[4] + value - sh[3]
                    digest.update(name.encode() + co[start:start + ssize])
                    found = True
        pos = fat.find(magic, pos + 1)
    return digest.hexdigest() if found else None


def pmc_fields(path, kernel, config):
    """HBM traffic and VALU issue of the render kernel from a committed rocprofv3 --pmc summary
    (scripts/pmc_json.py) of the same kernel, workload AND build (sha256 of the timed kernel's
    machine code and descriptor, kernel_sha256);
    (record, status) with record None when absent, mismatched or from another build."""
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, "absent"
    if rec.get("kernel") != kernel or rec.get("config") != config:
        return None, "other kernel or workload"
    here = kernel_sha256()
    if here is None:  # a timed kernel's symbol is missing from the loaded library
        return None, "timed kernel not found in the library"
    if rec.get("kernel_sha256") != here:
        return None, "stale: summary of another build of the timed kernel"
    return rec, "current build of the timed kernel"




# Issue cost of one wave64 VALU instruction per SIMD, cycles, by PMC class. NOMINAL: the ISA's
# rates on gfx950 (157.3 TF FP32 = 1024 SIMDs x 2.4 GHz x a wave64 FMA every 2 cycles;
# MI355X_MICROARCH.md): 2 for the f32/int32 classes and for the VALU count the typed counters
# leave over (compares, v_cndmask, conversions, min/max, DPP, moves), 4 for 64-bit integer, 8 for
# transcendentals (rcp, sqrt). UBENCH: as measured with 8 waves per SIMD (scripts/ubench_int.hip,
# profiles/r02/ubench_int.txt): plain ~2.4 (an SGPR operand, integer multiplies, bfe/add3 ~4.2),
# int64 ~4.2, trans ~8.2, the rest counted at ~4.2. The nominal count is the floor of the frame's
# VALU issue time; the ubench count overstates it (on config 3 it exceeds the frame period: the
# isolated rates include dependency stalls that other waves' issue hides in the kernel).
ISSUE_CYCLES_NOMINAL = {"plain": 2.0, "int64": 4.0, "trans": 8.0, "other": 2.0}
ISSUE_CYCLES_UBENCH = {"plain": 2.4, "int64": 4.2, "trans": 8.2, "other": 4.2}


def issue_roofline(pmc, ms_per_step):
    """The VALU issue roofline: sum over PMC instruction classes of count x
    issue cycles, over the issue capacity of one frame period (1024 SIMDs x the PMC run's clock
    x ms_per_step). issue_frac at the nominal rates, issue_frac_ubench at the measured ones."""
    c = pmc.get("counters", {})
    need = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32",
            "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_TRANS_F32")
    if any(k not in c for k in need):
        return {"issue_frac": None}
    plain = c["SQ_INSTS_VALU_ADD_F32"] + c["SQ_INSTS_VALU_MUL_F32"] + c["SQ_INSTS_VALU_FMA_F32"] + c["SQ_INSTS_VALU_INT32"]
    int64, trans = c["SQ_INSTS_VALU_INT64"], c["SQ_INSTS_VALU_TRANS_F32"]
    other = max(0.0, c["SQ_INSTS_VALU"] - plain - int64 - trans)
    cap = 1024 * pmc["clock_ghz"] * 1e9 * ms_per_step * 1e-3
    tot = c["SQ_INSTS_VALU"]

    def cycles(r):
        return plain * r["plain"] + int64 * r["int64"] + trans * r["trans"] + other * r["other"]

    nom, ub = cycles(ISSUE_CYCLES_NOMINAL), cycles(ISSUE_CYCLES_UBENCH)
    return {"issue_frac": round(nom / cap, 4), "issue_frac_ubench": round(ub / cap, 4),
            "issue_cycles_per_frame": round(nom), "valu_insts_per_frame": round(tot),
            "issue_mix": {"plain_f32_int32": round(plain / tot, 4), "int64": round(int64 / tot, 4),
                          "trans": round(trans / tot, 4), "other": round(other / tot, 4)},
            "issue_model": "wave64 VALU issue cycles per SIMD at the ISA's nominal rates: f32/int32 and the "
                           "untyped rest 2, int64 4, transcendental 8 (issue_frac, a floor); at the rates "
                           "measured in isolation 2.4 / 4.2 / 8.2 / 4.2 (issue_frac_ubench, an overstatement); "
                           "capacity = 1024 SIMDs x the PMC run's clock x ms_per_step"}


def dropin_timing(arrays, cam, W, H, spp, depth, seed, repeats=3):
    """The reference's entry as a caller meets it (cuda_impl, called once per frame at
    main.cxx:114 into the caller's vector of main.cxx:112): rt_render_rgb8 into a host buffer
    allocated once, through the synchronous C-ABI path (rt::render_impl's), timed on the host
    from call to return: the first call (scene build, workspaces, frame buffers) and repeats
    (the kept per-device context)."""
    import ctypes as C
    import numpy as np
    import raytracinginoneweekend_amd as rt
    from raytracinginoneweekend_amd import _abi as abi
    s, m = arrays
    s = np.ascontiguousarray(s, dtype=abi.SPHERE_DTYPE)
    m = np.ascontiguousarray(m, dtype=abi.MATERIAL_DTYPE)
    out = np.zeros((H, W, 3), dtype=np.uint8)
    p = rt.make_params(W, H, spp, depth, seed)
    rt.release_cached()

    def call():
        # no rt_stats, as rt::render_impl calls it (include/rt_render_impl.hpp): the product kernels
        t0 = time.perf_counter()
        rt._lib.check(rt.lib().rt_render_rgb8(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s),
                                              abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m), C.byref(cam.c),
                                              C.byref(p), abi.ptr(out, C.POINTER(C.c_uint8)), None))
        return (time.perf_counter() - t0) * 1e3

    first = call()
    rep = sorted(call() for _ in range(repeats))
    rt.release_cached()
    return {"dropin_first_ms": round(first, 3), "dropin_repeat_ms": round(rep[len(rep) // 2], 3),
            "dropin_repeat_all_ms": [round(x, 3) for x in rep],
            "dropin_entry": "rt_render_rgb8 (rt::render_impl's entry, no rt_stats): scene, render, u8 epilogue, "
                            "D2H into the caller's buffer; host clock call to return"}


def cpu_info():
    """(model, nproc, affinity cores, cores this job may use): the GPU box gives one GPU's job
    a share of the host (OMP_NUM_THREADS, 16 there) out of a larger affinity set."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return model, nproc, aff, max(1, min(aff, share))


def cpu_baseline(cfg, camera, seed, rows, threads):
    """The CPU baseline of BASELINE.md §4 on this host, on evenly spaced rows of the frame:
    - value: the REFERENCE's own CPU path (oracle/_ref/ref_harness_pcg, compiled from
      /root/reference: per-call std::vector + stable_partition + min_element,
      raytracer.hxx:100-117) on every core this job may use, rows interleaved over threads;
    - single_thread: the same binary on one thread (a smaller row sample);
    - optimized: the CPU restatement (oracle/rt_oracle.cpp: allocation-free closest hit, the
      same bits) on the same cores and rows."""
    scene, W, H, spp, depth = cfg
    model, nproc, aff, share = cpu_info()
    threads = threads or share
    step = max(1, H // rows)
    nrows = min(rows, (H + step - 1) // step)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_binding as O
    import raytracinginoneweekend_amd as rt
    host = {"cores": threads, "nproc": nproc, "affinity_cores": aff, "model": model}
    if scene == "cuda":  # the CUDA variant has no CPU path in the reference: the restatement
        s, m = rt.cuda_scene_arrays()
        p = O.make_params(W, H, spp, depth, 0, 0, step, nrows, flags=rt.abi.RT_FLAG_CUDA_COMPAT)
        t0 = time.perf_counter()
        O.render_cuda_compat(s, m, rt.Camera.cuda(W, H).c, p, threads=threads)
        sec = time.perf_counter() - t0
        return dict(value=round(W * nrows * spp / sec / 1e6, 4), unit="Mrays/s", kind="port",
                    sample=f"{nrows} rows (every {step}th) of {W}x{H}, {spp} spp, cuda_impl preset; {sec:.1f} s wall",
                    **host)
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness_pcg")
    if not os.path.exists(exe):
        raise SystemExit(f"cpu_baseline: {exe} is not built (oracle/build_ref.sh)")

    def ref_run(row_step, n, thr):
        cmd = [exe, "--scene", scene, "--scene-seed", "1234", "--w", str(W), "--h", str(H), "--spp", str(spp),
               "--depth", str(depth), "--seed", str(seed), "--camera", camera, "--row0", "0",
               "--row-step", str(row_step), "--rows", str(n), "--threads", str(thr), "--time"]
        out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
        return json.loads(out.strip().splitlines()[-1])

    r = ref_run(step, nrows, threads)
    n1 = max(1, nrows // 16)
    s1 = max(1, H // n1)
    r1 = ref_run(s1, n1, 1)
    s, m = rt.huge_scene_arrays(1234) if scene == "huge" else rt.simple_scene_arrays()
    cam = O.camera_default(W, H, 1 if camera == "corrected" else 0)
    p = O.make_params(W, H, spp, depth, seed, 0, step, nrows)
    t0 = time.perf_counter()
    O.render_f32(s, m, cam, p, threads=threads)
    so = time.perf_counter() - t0
    # The whole host: this job may use `threads` of the host's `aff` logical CPUs (the GPU box
    # allots 16 per GPU and its operators ask jobs to keep their worker pools to that share), so
    # the host-wide figure is the measured per-thread rate times every logical CPU: an upper
    # bound (SMT siblings share a core), stated as an estimate, not a measurement.
    whole = {"estimate": round(r["mrays_per_s"] / threads * aff, 2), "unit": "Mrays/s", "cores": aff,
             "basis": f"measured {r['mrays_per_s'] / threads:.4f} Mrays/s per thread on {threads} threads x {aff} "
                      "logical CPUs; linear in threads, an upper bound (SMT), not measured on all of them"}
    return dict(
        value=round(r["mrays_per_s"], 4), unit="Mrays/s", kind="reference", whole_host=whole,
        sample=f"{nrows} rows (every {step}th) of {W}x{H}, {spp} spp, {scene} scene, {camera} camera; "
               f"{r['seconds']:.1f} s wall; the rows' rate stands for the frame's (linear in rows)",
        single_thread={"value": round(r1["mrays_per_s"], 4), "cores": 1, "kind": "reference",
                       "sample": f"{n1} rows (every {s1}th); {r1['seconds']:.1f} s wall"},
        optimized={"value": round(W * nrows * spp / so / 1e6, 4), "cores": threads, "kind": "port",
                   "sample": f"same rows, the restatement oracle/rt_oracle.cpp; {so:.1f} s wall"},
        **host)


def launch_check(world, rank, local):
    """--launch-check: the rank joins a gloo group, agrees on the world with an all-reduce and
    prints one JSON line; no GPU call (tests/test_bench_launcher.py)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([rank], dtype=torch.int64)
        dist.all_reduce(t)
        total = int(t.item())
        dist.destroy_process_group()
    else:
        total = 0
    print(json.dumps({"launch_check": True, "rank": rank, "local_rank": local, "world": world,
                      "rank_sum": total, "master_addr": os.environ.get("MASTER_ADDR")}), flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process started with --gpus N: become the launcher of N ranks (before any HIP call)
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launch_check:
        return launch_check(world, rank, local)
    hw_env = os.environ.get("GPU_MAX_HW_QUEUES")
    if args.hw_queues > 0:  # before anything starts HIP: 8 queues -> 4 render streams
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import torch.distributed as dist

    distributed = world > 1
    torch.cuda.set_device(local)
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import raytracinginoneweekend_amd as rt
    scene_name, W, H, spp, depth = CONFIGS[args.config]
    compat = scene_name == "cuda"
    arrays = rt.huge_scene_arrays(1234) if scene_name == "huge" else (
        rt.cuda_scene_arrays() if compat else rt.simple_scene_arrays())
    n_spheres = len(arrays[0])
    from raytracinginoneweekend_amd.rowtiles import FrameGather, rank_params
    rehearse = args.rehearse_world if world == 1 and args.rehearse_world > 1 else 0
    params = rank_params(W, H, spp, rehearse or world, args.rehearse_rank if rehearse else rank, max_depth=depth,
                         seed=args.seed, scalar_scene=args.variant == "scalar", fast_math=args.variant == "fast",
                         brute_force=args.traversal == "brute", cuda_compat=compat,
                         wavefront=args.variant == "wavefront")
    if rehearse and args.rehearse_blocks:
        # contiguous blocks of H // N rows, the last rank taking the remainder
        blk = H // rehearse
        params.row_offset, params.row_stride = args.rehearse_rank * blk, 1
        params.num_rows = blk if args.rehearse_rank < rehearse - 1 else H - blk * (rehearse - 1)
    rows = params.num_rows
    dev = torch.device("cuda", local)
    opts = rt.parse_options(args.options, rt.default_options())
    ds = rt.DeviceScene(arrays, device=local, options=opts)
    tile = torch.empty((rows, W, 3), dtype=torch.float32, device=dev)
    rgb8 = args.output == "rgb8"
    tile8 = torch.empty((rows, W, 3), dtype=torch.uint8, device=dev) if rgb8 else None
    gather = FrameGather(tile8 if rgb8 else tile, world, rank, height=None if rehearse else H)
    seg = torch.zeros(3, dtype=torch.int64, device=dev)  # segments, sphere tests, box tests
    stream = torch.cuda.current_stream(dev)

    if rehearse and args.rehearse_gather:
        fake = torch.empty((rehearse, rows, W, 3), dtype=torch.float32, device=dev)
        frame_r = torch.empty((rows * rehearse, W, 3), dtype=torch.float32, device=dev)

    def out_frame():
        """rank 0's output of a step: the gathered frame (N > 1), the stood-in gathered frame of a
        rehearsal with --rehearse-gather (so its frame wall clock ends with the whole frame's copy
        to the host), or its own tile."""
        if rehearse and args.rehearse_gather:
            return frame_r
        return gather.frame if (world > 1 and not rehearse) else (tile8 if rgb8 else tile)

    # the reference's entry returns the frame in host memory (cuda_impl.cu:449-452): the frame
    # wall clock ends with the device->host copy into a pinned buffer
    host_frame = torch.empty(out_frame().shape, dtype=out_frame().dtype, pin_memory=True) if rank == 0 else None
    parity = {}
    # frames of the timed kernels this process renders (scripts/pmc_json.py divides its counters
    # by it: a frame is one pass alone, or several ring passes beside other frames)
    issued = [0]

    def measure(cam, steps, warmup, check_parity=False):
        """warmup untimed frames, then `steps` frames timed between barriers + syncs (max over
        ranks), then one frame alone three times on the device (its latency, median) and three
        times including the copy of the frame to host memory (the frame wall clock), then one
        frame of the counting kernel (the same paths and bits, plus tallies of segments and
        executed tests: the work of every frame of this workload, which the timed frames do not
        tally). check_parity: rank 0 compares the last timed frame with the reference's digests
        (outside the timed region)."""
        def step(count_segments):
            ds.render(cam, params, tile.data_ptr(), stream.cuda_stream, seg.data_ptr() if count_segments else None)
            issued[0] += 0 if count_segments else 1
            if rgb8:
                rt.epilogue_rgb8_device(tile.data_ptr(), tile8.data_ptr(), rows * W, stream.cuda_stream)
            if not rehearse:
                gather(tile8 if rgb8 else tile)
            elif args.rehearse_gather:
                # the peers' tiles landing in the gather buffer: one copy kernel, as RCCL's gather
                # receives them in one grouped operation; then the de-interleave, as FrameGather
                fake[1:].copy_(tile.unsqueeze(0).expand(rehearse - 1, *tile.shape))
                frame_r.view(rows, rehearse, W, 3).copy_(fake.transpose(0, 1))

        for _ in range(warmup):
            step(False)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(False)
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        spans = ds.kernel_times(steps)  # HIP-event spans of the timed frames' render launches
        if check_parity and rank == 0:
            # a rehearsal checks its own rows (the stood-in gather buffer holds copies of them)
            frame = (tile8 if rgb8 else tile).cpu().numpy() if rehearse else out_frame().cpu().numpy()
            off, stride = (0, 1) if not rehearse else (params.row_offset, params.row_stride)
            parity.update(parity_record(frame, args.config, W, H, off, stride, args.seed, args.camera,
                                        args.variant, args.output))
        lat, wall = [], []
        for _ in range(3):  # alternating, so both see the same clocks
            for to_host in (False, True):
                torch.cuda.synchronize()
                if distributed:
                    dist.barrier()
                t1 = time.perf_counter()
                step(False)
                if to_host and rank == 0:
                    host_frame.copy_(out_frame(), non_blocking=True)
                torch.cuda.synchronize()
                (wall if to_host else lat).append(time.perf_counter() - t1)
        latency, wall_clock = sorted(lat)[1], sorted(wall)[1]
        torch.cuda.synchronize()
        seg.zero_()
        step(True)
        torch.cuda.synchronize()
        counts = [int(x) * steps for x in seg.tolist()]  # per frame x timed frames
        counts_all = counts
        if distributed:
            t = torch.tensor([elapsed, latency, wall_clock], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, latency, wall_clock = float(t[0].item()), float(t[1].item()), float(t[2].item())
            sg = seg.clone()
            dist.all_reduce(sg)
            counts_all = [int(x) for x in sg.tolist()]
        return elapsed, (latency, wall_clock), spans, counts, counts_all

    def summary(elapsed, lat_wall, spans, counts, counts_all, steps):
        latency, wall_clock = lat_wall
        segments, sph_tests, box_tests = counts
        primaries = (W * rows if rehearse else W * H) * spp * steps
        period = elapsed / steps
        # executed work per frame on this rank: every ray-sphere test (20 FLOP)
        # and every cluster-box slab test (19 FLOP) the kernel ran
        flop_frame = (sph_tests * FLOP_PER_TEST + box_tests * FLOP_PER_BOX) / steps
        achieved = flop_frame / period / 1e12
        span = sum(spans) / max(len(spans), 1)
        return {
            "value": primaries / elapsed / 1e6, "ms_per_step": period * 1e3, "frame_latency_ms": latency * 1e3,
            "frame_wall_ms": wall_clock * 1e3,
            "segments_per_primary": counts_all[0] / primaries,
            "msegments_per_s": counts_all[0] / elapsed / 1e6,
            "gtests_per_s": counts_all[1] / elapsed / 1e9, "gbox_tests_per_s": counts_all[2] / elapsed / 1e9,
            "tests_per_segment": sph_tests / max(segments, 1), "boxes_per_segment": box_tests / max(segments, 1),
            "flop_per_frame": flop_frame, "achieved": achieved,
            # the reference's brute force: every segment tests every sphere
            "effective_tflops": segments / steps * n_spheres * FLOP_PER_TEST / period / 1e12,
            "span_ms": span, "span_achieved": flop_frame / (span * 1e-3) / 1e12 if span else None,
        }

    mode = rt.CORRECTED if args.camera == "corrected" else rt.REFERENCE
    cam = rt.Camera.cuda(W, H) if compat else rt.Camera.default(W, H, mode)
    main_m = summary(*measure(cam, args.steps, args.warmup, check_parity=not compat), args.steps)
    usage = ds.usage()  # the cut of the timed frames (before the corrected-camera frames)
    corr = None
    if args.corrected_steps > 0 and not compat and args.camera == "reference":
        # the representative path-tracing load (7 segments per primary): the corrected camera
        # (direction - origin) on the same workload, a few frames after the headline ones
        corr = summary(*measure(rt.Camera.default(W, H, rt.CORRECTED), args.corrected_steps, 1),
                       args.corrected_steps)
    if rank == 0:
        r3 = lambda x: round(x, 3) if x is not None else None  # noqa: E731
        rec = {
            "metric": "Mrays/sec + frame wall-clock, huge-scene 1280x720x128spp @1/2/4/8 GPU",
            "value": round(main_m["value"], 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": r3(main_m["ms_per_step"]),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference huge scene, std::mt19937 seed 1234; per-sample PCG32 seed %d)" % args.seed,
            "config": {"workload": WORKLOAD[args.config], "scene": f"{scene_name} ({n_spheres} spheres)",
                       "width": W, "height": H, "spp": spp, "max_depth": depth, "camera": args.camera,
                       "kernel": "compat_kernel (cuda_impl.cu semantics, bit-exact vs its restatement)" if compat else
                       ("fast (FMA, stated tolerance)" if args.variant == "fast" else f"{args.variant} (bit-exact)")
                       + f", {args.traversal}", "parallelism": f"row-interleaved x{world}, RCCL gather of "
                       + ("u8 (gamma epilogue per rank)" if rgb8 else "f32") + " tiles",
                       "output": args.output, "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "hw_queues_env": hw_env,
                       # the scene's rt_options (library defaults, RT_OPTIONS, --options): deep-path
                       # split and the lone-pass size below which passes are not split
                       "deep_split": opts.deep_split, "deep_min_items": opts.deep_min_items,
                       "options": {k: getattr(opts, k) for k, _ in rt.abi.RtOptions._fields_ if k != "size"}},
            # ms_per_step is the steady-state period of a frame stream (frames in flight);
            # frame_wall_ms is ONE frame alone, start to finish, ending with the frame in host
            # memory as the reference's entry returns it (render, accumulate, gather, D2H copy
            # into pinned memory); frame_device_ms is the same frame without the copy (the
            # round-2 "frame_wall_ms"/"frame_latency_ms")
            "frame_wall_ms": r3(main_m["frame_wall_ms"]),
            "frame_device_ms": r3(main_m["frame_latency_ms"]),
            "frame_latency_ms": r3(main_m["frame_latency_ms"]),
            # render streams the timed frames rotated over (frames in flight), the workspaces and
            # the samples per pass (rt_scene_usage_get after the run)
            "frames_in_flight": usage["render_streams"], "workspaces": usage["workspaces"], "frames_issued": issued[0],
            "pass_samples": usage["pass_samples"],
            # device memory the scene held for the timed frames: HBM footprint of the product
            # (scene blobs, counters, slot workspaces, deep-path queues), and the workspaces alone
            "hbm_footprint_bytes": usage["device_bytes"], "hbm_workspace_bytes": usage["workspace_bytes"],
            "segments_per_primary": round(main_m["segments_per_primary"], 4),
            "msegments_per_s": round(main_m["msegments_per_s"], 1),
            "gtests_per_s": round(main_m["gtests_per_s"], 2),
            "gbox_tests_per_s": round(main_m["gbox_tests_per_s"], 2),
            "tests_per_segment": round(main_m["tests_per_segment"], 2),
            "boxes_per_segment": round(main_m["boxes_per_segment"], 2),
            "roofline": {
                "bound": "valu", "achieved": r3(main_m["achieved"]), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(main_m["achieved"] / PEAK_FP32_TFLOPS, 4), "traffic": None,
                "kernel": "compat_kernel" if compat else "render_kernel",
                "work": "executed ray-sphere tests x 20 FLOP + cluster-box tests x 19 FLOP per frame, over the "
                        "frame period (ms_per_step)",
                "flop_per_frame": main_m["flop_per_frame"],
                # brute-force equivalent (segments x spheres x 20 FLOP over the period): a speed-up
                # figure over the reference's algorithm, NOT a fraction of any peak
                "effective_tflops": round(main_m["effective_tflops"], 2),
                # a frame's render launches overlap other frames' (frames in flight): their
                # HIP-event span is a latency, shown for reference only
                "per_launch_span_ms": r3(main_m["span_ms"]),
                "per_launch_span_achieved": r3(main_m["span_achieved"]),
            },
        }
        v = {"exact": 0, "scalar": 1, "fast": 2, "wavefront": 0}[args.variant]
        cull = 0 if args.traversal == "brute" or v == 1 else 7
        kname = TIMED_KERNEL_NAMES if (v, cull) == (0, 7) else f"render_kernel<{v}, {cull}, false, false, false>"
        pmc, status = pmc_fields(args.pmc, kname, {"workload": WORKLOAD[args.config], "camera": args.camera,
                                                   "traversal": args.traversal, "n_gpus": world})
        if args.variant == "wavefront":  # other kernels did the work: no render_kernel PMC
            pmc, status = None, "other kernels (wave_gen_kernel, wave_bounce_kernel)"
        rec["roofline"]["pmc_status"] = status
        if pmc and not rehearse:
            # HBM bytes per frame (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE, one
            # launch per frame here) and the VALU issue, from the PMC summary of THIS build
            rec["roofline"]["traffic"] = pmc["hbm_bytes_per_frame"]
            rec["roofline"]["traffic_unit"] = "bytes/frame"
            rec["roofline"]["valu_insts_per_frame"] = pmc["valu_insts"]
            # VALU pipe busy over the frame period: wave64 VALU = 2 cycles, 1024 SIMDs (a floor)
            rec["roofline"]["valu_busy"] = round(
                pmc["valu_insts"] * 2.0 / (1024 * pmc["clock_ghz"] * 1e9 * main_m["ms_per_step"] * 1e-3), 4)
            rec["roofline"].update(issue_roofline(pmc, main_m["ms_per_step"]))
            rec["roofline"]["pmc_source"] = os.path.relpath(args.pmc, REPO)
        if parity:
            rec["parity"] = parity
        if corr:
            rec["corrected_camera"] = {
                "value": round(corr["value"], 3), "unit": "Mrays/s", "steps": args.corrected_steps,
                "ms_per_step": r3(corr["ms_per_step"]), "frame_latency_ms": r3(corr["frame_latency_ms"]),
                "segments_per_primary": round(corr["segments_per_primary"], 4),
                "msegments_per_s": round(corr["msegments_per_s"], 1), "gtests_per_s": round(corr["gtests_per_s"], 2),
                "roofline_achieved": r3(corr["achieved"]), "roofline_frac": round(corr["achieved"] / PEAK_FP32_TFLOPS, 4),
                "effective_tflops": round(corr["effective_tflops"], 2)}
        if rehearse:
            rr = args.rehearse_rank
            rows_desc = (f"rows {params.row_offset}..{params.row_offset + rows - 1}" if args.rehearse_blocks
                         else f"rows {rr}, {rr + rehearse}, ... ({rows} rows)")
            rec["rehearsal"] = (f"rank {rr} of {rehearse}: {rows_desc}, "
                                + ("gather's device copies stood in on the caller stream" if args.rehearse_gather
                                   else "no gather") + "; value = "
                                f"this rank's Mrays/s, x{rehearse} for the ideal {rehearse}-GPU job")
            if args.rehearse_gather:
                # the N-GPU frame as one rank sees it, REHEARSED ON ONE GPU, NOT MEASURED: its share's
                # lone frame with the gather's device work stood in (the N-1 peer tiles copied into
                # the gather buffer, the de-interleave) and the whole frame copied to host memory,
                # plus the peers' tiles over xGMI, which one GPU cannot run: each peer sends its
                # tile on its own link at once, estimated at 50 GB/s per link
                tile_bytes = rows * W * (3 if rgb8 else 12)
                xgmi_ms = tile_bytes / 50e9 * 1e3
                rec["rehearsal_projection"] = {
                    "n_gpus": rehearse, "share_period_ms": r3(main_m["ms_per_step"]),
                    "share_frame_wall_ms": r3(main_m["frame_wall_ms"]),
                    "xgmi_tile_bytes": tile_bytes, "xgmi_estimate_ms": round(xgmi_ms, 4),
                    "projected_frame_wall_ms": r3(main_m["frame_wall_ms"] + xgmi_ms),
                    "note": "rehearsed on one GPU, not measured: rank 0's rows alone, the gather's device copies "
                            "and the full-frame D2H copy stood in; xGMI transfer time estimated"}
        if world == 1 and not rehearse and not compat and args.variant == "exact" and args.traversal == "cull" \
                and not args.no_dropin:
            rec.update(dropin_timing(arrays, cam, W, H, spp, depth, args.seed))
        if world == 1 and not args.no_cpu_baseline and not rehearse:
            rec["cpu_baseline"] = cpu_baseline(CONFIGS[args.config], args.camera, args.seed, args.cpu_rows,
                                               args.cpu_threads)
        print(json.dumps(rec), flush=True)
    ds.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
