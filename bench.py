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

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

The cpu_baseline leg (rank 0, N=1) times the REFERENCE's own CPU path (oracle/_ref, built
from /root/reference) on a bounded row subset of the same workload, on this host's cores.
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
    ap.add_argument("--variant", default="exact", choices=["exact", "fast", "scalar"],
                    help="exact: bit-exact kernel; fast: FMA kernel within the stated tolerance; "
                         "scalar: brute-force scalar-cache A/B")
    ap.add_argument("--traversal", default="cull", choices=["cull", "brute"],
                    help="cull: exact cluster culling (same bits); brute: every sphere, as the reference")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rows", type=int, default=240, help="rows in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--rehearse-world", type=int, default=0,
                    help="diagnostic, 1 GPU: render only rank 0's rows of an N-way split (no gather) to "
                         "estimate one rank's frame time at N GPUs; not a bench line")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts; 0 = leave the environment): "
                         "the library runs one render stream fewer than this, 2..4 (rt_host.cpp pipeline_env)")
    ap.add_argument("--rehearse-gather", action="store_true",
                    help="with --rehearse-world N: stand in for rank 0's gather with its device work on the "
                         "caller stream (the N-1 peer tiles copied into the gather buffer, then the "
                         "de-interleave copy), to see whether that work waits for CU slots")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_render_c3.json"),
                    help="PMC summary of this kernel (scripts/pmc_round.sh) for roofline.traffic / VALU busy")
    return ap.parse_args()


def pmc_fields(path, kernel, config):
    """HBM traffic and VALU issue of the render kernel from a committed rocprofv3 --pmc summary
    (scripts/pmc_json.py) of the same kernel and workload; None when absent or mismatched."""
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if rec.get("kernel") != kernel or rec.get("config") != config:
        return None
    return rec


def frames_in_flight():
    """Render streams (RT_PIPELINE, rt_host.cpp pipeline_env: by default GPU_MAX_HW_QUEUES - 1,
    within 2..4)."""
    v = os.environ.get("RT_PIPELINE", "")
    if v:
        return max(1, min(int(v), 4))
    return max(2, min(int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) - 1, 4))


def cpu_baseline(cfg, camera, seed, rows, threads):
    """Reference CPU path (oracle/_ref/ref_harness_pcg) on `rows` evenly spaced rows."""
    scene, W, H, spp, depth = cfg
    step = max(1, H // rows)
    nrows = min(rows, (H + step - 1) // step)
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", 0)) or min(16, os.cpu_count() or 1)
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness_pcg")
    sample = f"{nrows} rows (every {step}th) of {W}x{H}, {spp} spp, {scene} scene, {camera} camera"
    if scene == "cuda":  # the CUDA variant has no CPU path in the reference: the restatement
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_binding as O
        import raytracinginoneweekend_amd as rt
        s, m = rt.cuda_scene_arrays()
        p = O.make_params(W, H, spp, depth, 0, 0, step, nrows, flags=rt.abi.RT_FLAG_CUDA_COMPAT)
        t0 = time.perf_counter()
        O.render_cuda_compat(s, m, rt.Camera.cuda(W, H).c, p, threads=threads)
        sec = time.perf_counter() - t0
        return {"value": round(W * nrows * spp / sec / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
                "sample": f"{nrows} rows (every {step}th) of {W}x{H}, {spp} spp, cuda_impl preset; {sec:.1f} s wall"}
    if os.path.exists(exe):
        cmd = [exe, "--scene", scene, "--scene-seed", "1234", "--w", str(W), "--h", str(H), "--spp", str(spp),
               "--depth", str(depth), "--seed", str(seed), "--camera", camera, "--row0", "0",
               "--row-step", str(step), "--rows", str(nrows), "--threads", str(threads), "--time"]
        out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
        return {"value": round(r["mrays_per_s"], 4), "unit": "Mrays/s", "cores": threads, "kind": "reference",
                "sample": sample + f"; {r['seconds']:.1f} s wall"}
    # fallback: the CPU restatement (bit-identical to the reference, tests/test_oracle_golden.py)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import numpy as np
    import oracle_binding as O
    import raytracinginoneweekend_amd as rt
    s, m = rt.huge_scene_arrays(1234) if scene == "huge" else rt.simple_scene_arrays()
    cam = O.camera_default(W, H, 1 if camera == "corrected" else 0)
    p = O.make_params(W, H, spp, depth, seed, 0, step, nrows)
    t0 = time.perf_counter()
    O.render_f32(s, m, cam, p, threads=threads)
    sec = time.perf_counter() - t0
    del np
    return {"value": round(W * nrows * spp / sec / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": sample + f"; {sec:.1f} s wall"}


def main():
    args = parse()
    if args.hw_queues > 0:  # before anything starts HIP
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes")
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
    mode = rt.CORRECTED if args.camera == "corrected" else rt.REFERENCE
    cam = rt.Camera.cuda(W, H) if compat else rt.Camera.default(W, H, mode)
    from raytracinginoneweekend_amd.rowtiles import FrameGather, rank_params
    rehearse = args.rehearse_world if world == 1 and args.rehearse_world > 1 else 0
    params = rank_params(W, H, spp, rehearse or world, rank, max_depth=depth, seed=args.seed,
                         scalar_scene=args.variant == "scalar", fast_math=args.variant == "fast",
                         brute_force=args.traversal == "brute", cuda_compat=compat)
    rows = params.num_rows
    dev = torch.device("cuda", local)
    ds = rt.DeviceScene(arrays, device=local)
    tile = torch.empty((rows, W, 3), dtype=torch.float32, device=dev)
    gather = FrameGather(tile, world, rank)
    seg = torch.zeros(3, dtype=torch.int64, device=dev)  # segments, sphere tests, box tests
    stream = torch.cuda.current_stream(dev)

    if rehearse and args.rehearse_gather:
        fake = torch.empty((rehearse, rows, W, 3), dtype=torch.float32, device=dev)
        frame_r = torch.empty((rows * rehearse, W, 3), dtype=torch.float32, device=dev)

    def step(count_segments):
        ds.render(cam, params, tile.data_ptr(), stream.cuda_stream, seg.data_ptr() if count_segments else None)
        if not rehearse:
            gather(tile)
        elif args.rehearse_gather:
            for r in range(1, rehearse):  # one copy kernel per peer, as the gather's receives
                fake[r].copy_(tile)
            frame_r.view(rows, rehearse, W, 3).copy_(fake.transpose(0, 1))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    seg.zero_()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kt = ds.kernel_times(args.steps)  # render-kernel durations of the timed steps (HIP events)
    # one frame alone (no frame in flight beside it): its latency, median of 3
    lat = []
    for _ in range(3):
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        t1 = time.perf_counter()
        step(False)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t1)
    latency = sorted(lat)[1]
    if distributed:
        t = torch.tensor([latency], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        latency = float(t.item())
    segments, sph_tests, box_tests = [int(x) for x in seg.tolist()]
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        sg = seg.clone()
        dist.all_reduce(sg)
        segments_all = int(sg[0].item())
    else:
        segments_all = segments

    primaries = W * rows * spp * args.steps if rehearse else W * H * spp * args.steps
    value = primaries / elapsed / 1e6
    # roofline of the dominant kernel (render_kernel) on this rank
    k_avg_ms = sum(kt) / len(kt)
    # executed work: every ray-sphere test the kernel ran (20 FLOP) + every cluster AABB test
    # (19 FLOP); brute force executes segments x n_spheres tests
    flop_per_launch = (sph_tests * FLOP_PER_TEST + box_tests * FLOP_PER_BOX) / args.steps
    achieved = flop_per_launch / (k_avg_ms * 1e-3) / 1e12
    # consecutive launches overlap (frames in flight, half grids while others run), so a
    # launch's own duration is longer than its share of the GPU: the same work per frame over
    # the steady-state frame period is the throughput view
    achieved_stream = flop_per_launch / (elapsed / args.steps) / 1e12
    brute_equiv = segments / args.steps * n_spheres * FLOP_PER_TEST / (k_avg_ms * 1e-3) / 1e12
    if rank == 0:
        rec = {
            "metric": "Mrays/sec + frame wall-clock, huge-scene 1280x720x128spp @1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference huge scene, std::mt19937 seed 1234; per-sample PCG32 seed %d)" % args.seed,
            "config": {"workload": WORKLOAD[args.config], "scene": f"{scene_name} ({n_spheres} spheres)",
                       "width": W, "height": H, "spp": spp, "max_depth": depth, "camera": args.camera,
                       "kernel": "compat_kernel (cuda_impl.cu semantics, bit-exact vs its restatement)" if compat else
                       ("fast (FMA, stated tolerance)" if args.variant == "fast" else f"{args.variant} (bit-exact)")
                       + f", {args.traversal}", "parallelism": f"row-interleaved x{world}, RCCL gather",
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))},
            "frame_wall_ms": round(elapsed / args.steps * 1e3, 3),
            "frame_latency_ms": round(latency * 1e3, 3),
            "frames_in_flight": frames_in_flight(),
            "segments_per_primary": round(segments_all / primaries, 4),
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": None,
                         "kernel": "compat_kernel" if compat else "render_kernel", "kernel_avg_ms": round(k_avg_ms, 3),
                         "flop_per_launch": flop_per_launch, "work": "executed sphere+box tests",
                         "brute_force_equiv_tflops": round(brute_equiv, 2),
                         "achieved_frame_stream": round(achieved_stream, 3),
                         "frac_frame_stream": round(achieved_stream / PEAK_FP32_TFLOPS, 4)},
            "tests_per_segment": round(sph_tests / max(segments, 1), 2),
            "kernel_tests_per_s": round(sph_tests / args.steps / (k_avg_ms * 1e-3) / 1e12, 4),
            "boxes_per_segment": round(box_tests / max(segments, 1), 2),
        }
        v = {"exact": 0, "scalar": 1, "fast": 2}[args.variant]
        cull = 0 if args.traversal == "brute" or v == 1 else 7
        kname = f"render_kernel<{v}, {cull}, false>"
        pmc = pmc_fields(args.pmc, kname, {"workload": WORKLOAD[args.config], "camera": args.camera,
                                            "traversal": args.traversal, "n_gpus": world})
        if pmc and not rehearse:
            # HBM bytes per launch (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE) and
            # the VALU issue fraction, from the committed PMC summary of this kernel
            rec["roofline"]["traffic"] = pmc["hbm_bytes_per_launch"]
            rec["roofline"]["traffic_unit"] = "bytes/launch"
            rec["roofline"]["valu_busy"] = pmc["valu_busy"]
            # the same VALU instructions per frame over the steady-state frame period (launches
            # overlap there; valu_busy above divides by one serialized dispatch's duration)
            rec["roofline"]["valu_busy_frame_stream"] = round(
                pmc["valu_insts"] * 2.0 / (1024 * pmc["clock_ghz"] * 1e9 * elapsed / args.steps), 4)
            rec["roofline"]["pmc_source"] = os.path.relpath(args.pmc, REPO)
        if rehearse:
            rec["rehearsal"] = (f"rank 0 of {rehearse}: rows 0, {rehearse}, ... ({rows} rows), "
                                + ("gather's device copies stood in on the caller stream" if args.rehearse_gather
                                   else "no gather") + "; value = "
                                f"this rank's Mrays/s, x{rehearse} for the ideal {rehearse}-GPU job")
        if world == 1 and not args.no_cpu_baseline and not rehearse:
            rec["cpu_baseline"] = cpu_baseline(CONFIGS[args.config], args.camera, args.seed, args.cpu_rows,
                                               args.cpu_threads)
        print(json.dumps(rec), flush=True)
    ds.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
