"""GPU parity of whole frames at the BASELINE sizes and of the frame-level entry points:
configs 4 and 5 (multi-pass frames) against the reference's golden rows and the oracle, the
persistent multi-GPU context (rt_multi_*) with virtual ranks on one device, the u8 gather,
the PPM writer, and renders whose caller stream changes between calls.

Tolerance: f32 bitwise (0 ULP), as tests/test_gpu_parity.py; u8 within 1 LSB on a handful of
texels (device pow vs glibc powf).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import golden_io as G
import oracle_binding as O
import raytracinginoneweekend_amd as rt
from raytracinginoneweekend_amd import _abi as abi

pytestmark = pytest.mark.gpu


def _bits_equal(a, b, what=""):
    a = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    b = np.ascontiguousarray(b, dtype=np.float32).view(np.uint32)
    bad = np.count_nonzero(a != b)
    assert bad == 0, f"{what}: {bad} of {a.size} values differ"


def _u8_close(a, b):
    d = np.abs(a.astype(np.int16) - b.astype(np.int16))
    assert d.max() <= 1
    assert np.count_nonzero(d) <= max(2, a.size // 10000)


# ---- configs 4 and 5: the full multi-pass frames ------------------------------------------
# One pass holds a multiple of 4 samples within the 2 GiB slot workspace: config 4 (3840x2160,
# 99.5 MB per sample) runs 13 passes of 20 samples (the last 16), config 5 (1280x720, 11 MB
# per sample) 6 passes of 192 (the last 64). Every pass's partial sums are carried in the
# accumulation buffer, passes rotate over the render streams and workspaces; the frame must
# equal the reference's blocked reduce over all samples (src/main.cxx:191-215).
FULL = {
    "c4": dict(W=3840, H=2160, spp=256, golden="c4_huge_3840x2160_row1133_s256", rows=[0, 1079, 2159]),
    "c5": dict(W=1280, H=720, spp=1024, golden="c5_huge_1280x720_row377_s1024", rows=[0, 719]),
}


def _full_ref(cfg):
    """The reference's whole-frame digests (tests/golden/make_fullframe.py)."""
    with open(os.path.join(G.GOLDEN, "fullframe.json")) as f:
        return json.load(f)[cfg]


def _assert_frame_digest(img, ref, what):
    """Whole f32 frame == the reference's, bit for bit; on a mismatch name the rows."""
    got = hashlib.sha256(np.ascontiguousarray(img, dtype=np.float32).tobytes()).hexdigest()
    if got != ref["sha256_f32"]:
        bad = [y for y in range(img.shape[0])
               if hashlib.sha256(img[y].tobytes()).hexdigest()[:16] != ref["row_sha256_16"][y]]
        raise AssertionError(f"{what}: frame differs from the reference in {len(bad)} of {img.shape[0]} rows, "
                             f"first {bad[:8]}")


# ---- configs 2 and 3 (the headline) whole, through the bench's frames-in-flight path -------
@pytest.mark.parametrize("cfg", ["c3", "c2"])
def test_baseline_frame_stream_matches_reference(cfg):
    """BASELINE configs 3 (huge scene 1280x720 @128 spp, the bench's workload) and 2 (simple
    scene 1280x720 @64 spp, depth 50), rendered as bench.py renders them: DeviceScene.render
    into device buffers, frames back to back on one stream without host sync (renders on the
    internal streams, partial grids while others run, the deep-path split at its defaults,
    two-part accumulation for the lone first frame), then a counting frame. Every frame's
    whole f32 image must equal the reference's own render of the full frame
    (oracle/_ref/ref_harness_pcg, src/main.cxx:185-215), compared by sha256."""
    torch = pytest.importorskip("torch")
    ref = _full_ref(cfg)
    W, H, spp, depth = ref["width"], ref["height"], ref["spp"], ref["depth"]
    s, m = G.scene(ref["scene"])
    ds = rt.DeviceScene((s, m))
    p = rt.make_params(W, H, spp, depth, ref["seed"])
    cam = rt.Camera.default(W, H)
    stream = torch.cuda.current_stream().cuda_stream
    outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(5)]
    seg = torch.zeros(3, dtype=torch.int64, device="cuda")
    for k, o in enumerate(outs):
        ds.render(cam, p, o.data_ptr(), stream, seg.data_ptr() if k == len(outs) - 1 else None)
    torch.cuda.synchronize()
    ds.close()
    for k, o in enumerate(outs):
        _assert_frame_digest(o.cpu().numpy(), ref, f"{cfg} frame {k}")
    assert int(seg[0]) > W * H * spp  # every primary plus its bounces


@pytest.mark.parametrize("share", [(2, 1), (4, 2), (8, 0), (8, 7)])
def test_config3_row_shares_match_reference_rows(share):
    """Config 3's row shares as bench.py --gpus N renders them (rank r: rows r, r + N, ...): each
    row of a share must equal the reference's row (its sha256 in tests/golden/fullframe.json):
    the tile classes and the sky proof over strided rows (row_offset, row_stride), the sky
    kernel's pixel enumeration through the share's block permutation, a lone frame (its main
    launch leaving room for the sky kernel on the next render stream), then two back to back."""
    torch = pytest.importorskip("torch")
    n, r = share
    ref = _full_ref("c3")
    W, H, spp, depth = ref["width"], ref["height"], ref["spp"], ref["depth"]
    s, m = G.scene(ref["scene"])
    rows = (H - r + n - 1) // n
    p = rt.make_params(W, H, spp, depth, ref["seed"], row_offset=r, row_stride=n, num_rows=rows)
    cam = rt.Camera.default(W, H)
    ds = rt.DeviceScene((s, m))
    stream = torch.cuda.current_stream().cuda_stream
    outs = [torch.empty((rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(3)]
    ds.render(cam, p, outs[0].data_ptr(), stream)
    torch.cuda.synchronize()
    sky = ds.usage()["sky_tiles"]
    for o in outs[1:]:
        ds.render(cam, p, o.data_ptr(), stream)
    torch.cuda.synchronize()
    ds.close()
    assert sky > 0
    for k, o in enumerate(outs):
        img = o.cpu().numpy()
        bad = [i for i in range(rows)
               if hashlib.sha256(img[i].tobytes()).hexdigest()[:16] != ref["row_sha256_16"][r + i * n]]
        assert not bad, f"share {r}/{n} frame {k}: rows differ from the reference: {[r + i * n for i in bad[:8]]}"


def test_bounds_checked_frame_stream_c3():
    """Round 4's hipErrorIllegalAddress, pinned. The instrumented kernel
    (options stats=True) checks every lane-computed index into the scene blob, the sample slots
    and the deep queue before it uses it, and starts every lane's walk-shortcut neighbour word
    at 0x3fffffff (slots past any blob), as a stale or never-written word may hold. Over the
    config-3 frame stream (a lone first frame with its 8-wave deep launch, then frames in flight
    with 4-wave deep launches and global shading records) no index passes its bound, and the
    frames equal the reference's. With unbounded_nb the neighbour slots are formed without the
    lane's own bound, as before fd383c3: the check then reports them (and reads slot 0 instead,
    so the frames are unchanged) — the bound is what keeps those reads inside the blob."""
    torch = pytest.importorskip("torch")
    ref = _full_ref("c3")
    W, H, spp, depth = ref["width"], ref["height"], ref["spp"], ref["depth"]
    s, m = G.scene(ref["scene"])
    p = rt.make_params(W, H, spp, depth, ref["seed"])
    cam = rt.Camera.default(W, H)
    stream = torch.cuda.current_stream().cuda_stream
    for unbounded in (False, True):
        ds = rt.DeviceScene((s, m), options=rt.options(rt.default_options(), stats=True, unbounded_nb=unbounded))
        outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(3)]
        for o in outs:
            ds.render(cam, p, o.data_ptr(), stream)
        torch.cuda.synchronize()
        if unbounded:
            with pytest.raises(rt.RtError, match="neighbour slot"):
                ds.debug_counters()
        else:
            c = ds.debug_counters()
            assert c["wave_iters"] > 0
        ds.close()
        for k, o in enumerate(outs):
            _assert_frame_digest(o.cpu().numpy(), ref, f"c3 instrumented frame {k} (unbounded_nb={unbounded})")


@pytest.mark.parametrize("cfg", sorted(FULL))
def test_full_config_frame_matches_reference_rows(cfg):
    c = FULL[cfg]
    W, H, spp = c["W"], c["H"], c["spp"]
    s, m = G.scene("huge")
    img, st = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 1234, full_frame=True))
    assert st.primaries == W * H * spp
    # the whole frame against the reference's own full render (its digest must be committed:
    # tests/golden/make_fullframe.py; a missing digest fails)
    _assert_frame_digest(img, _full_ref(cfg), cfg)
    # the reference's own row (tests/golden/make_golden.py, oracle/_ref)
    meta, f32, u8 = G.render(c["golden"])
    y = meta["row_offset"]
    _bits_equal(img[y:y + 1], f32, f"{cfg} golden row {y}")
    _u8_close(O.epilogue_rgb8(img[y:y + 1]), u8)
    # further rows against the restatement (pinned to the reference by test_oracle_golden)
    cam = O.camera_default(W, H)
    for y in c["rows"]:
        ref, _ = O.render_f32(s, m, cam, rt.make_params(W, H, spp, 64, 1234, row_offset=y, num_rows=1),
                              threads=os.cpu_count())
        _bits_equal(img[y:y + 1], ref, f"{cfg} row {y}")
    # size-independent properties of the whole frame: finite, in [0, 1], every pixel written,
    # the reference camera's segment count (1.40 per primary on the huge scene)
    assert np.isfinite(img).all() and img.min() >= 0.0 and img.max() <= 1.0
    assert (img.reshape(-1, 3).max(axis=1) > 0).mean() > 0.99
    assert 1.35 < st.segments / st.primaries < 1.45


# ---- the persistent multi-GPU context ----------------------------------------------------
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_multi_context_virtual_ranks_match_single(n):
    """rt_multi_* with n ranks that all live on device 0 (tiles moved by device copies where
    RCCL would send/recv): the same tile layout, gather buffer and de-interleave as on n GPUs.
    f32 and u8 frames equal the single render, for ragged tiles (H % n != 0), several frames
    through one context, frame sizes that grow and shrink."""
    s, m = G.scene("huge")
    ctx = rt.MultiContext((s, m), devices=[0] * n)
    assert ctx.n_ranks == n and not ctx.uses_rccl
    for (W, H, spp, seed, mode) in [(64, 37, 4, 5, 0), (96, 50, 3, 6, 1), (40, 9, 5, 7, 0)]:
        cam = rt.Camera.default(W, H, mode)
        p = rt.make_params(W, H, spp, 64, seed)
        single, st1 = rt.render_f32((s, m), p, cam)
        got, stm = ctx.render_f32(p, cam)
        _bits_equal(got, single, f"n={n} {W}x{H}")
        assert stm.segments == st1.segments and stm.primaries == st1.primaries
        got8, _ = ctx.render_rgb8(p, cam)
        single8, _ = rt.render_rgb8((s, m), p, cam)
        np.testing.assert_array_equal(got8, single8)  # the same device epilogue on the same bits
    ctx.close()


def test_multi_context_streams_frames_without_sync():
    """Frames enqueued back to back on one stream through rt_multi_render_device (no host
    sync between them, tiles and gather buffer reused while earlier frames are in flight)
    land in stream order, each equal to its serial render."""
    torch = pytest.importorskip("torch")
    s, m = G.scene("huge")
    W, H = 48, 30
    ctx = rt.MultiContext((s, m), devices=[0, 0, 0, 0])
    jobs = [(rt.make_params(W, H, 8, 64, 1), rt.Camera.default(W, H, 0), False),
            (rt.make_params(W, H, 5, 64, 2), rt.Camera.default(W, H, 1), True),
            (rt.make_params(W, H, 12, 7, 3), rt.Camera.default(W, H, 0), False),
            (rt.make_params(W, H, 4, 64, 4), rt.Camera.default(W, H, 1), True)] * 2
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for p, cam, u8 in jobs:
        outs.append(torch.empty((H, W, 3), dtype=torch.uint8 if u8 else torch.float32, device="cuda"))
        ctx.render_device(cam, p, outs[-1].data_ptr(), stream, rgb8=u8)
    torch.cuda.synchronize()
    for (p, cam, u8), o in zip(jobs, outs):
        if u8:
            want, _ = rt.render_rgb8((s, m), p, cam)
            np.testing.assert_array_equal(o.cpu().numpy(), want)
        else:
            want, _ = rt.render_f32((s, m), p, cam)
            _bits_equal(o.cpu().numpy(), want)
    ctx.close()


def test_render_multi_rgb8_matches_golden():
    """rt_render_multi_rgb8 (u8 epilogue per rank, 3-byte gather) on config 1: within 1 LSB of
    the reference's u8 frame; equal to the single-device u8 render."""
    meta, _, u8 = G.render("c1_simple_200x100_s1")
    s, m = G.scene("simple")
    p = rt.make_params(meta["width"], meta["height"], meta["spp"], meta["depth"], meta["seed"])
    got, st = rt.render_multi_rgb8((s, m), p)
    _u8_close(got, u8)
    single, _ = rt.render_rgb8((s, m), p)
    np.testing.assert_array_equal(got, single)
    assert st.primaries == meta["width"] * meta["height"]


def test_ppm_of_gpu_frame_matches_reference_ppm(tmp_path):
    """app::save_to_file's P6 file for config 1, written by the reference (golden .ppm) and by
    rt_write_ppm from the GPU's u8 frame: identical header and size, texels within 1 LSB."""
    meta, _, _ = G.render("c1_simple_200x100_s1")
    ref = open(os.path.join(G.GOLDEN, meta["ppm"]), "rb").read()
    s, m = G.scene("simple")
    img, _ = rt.render_rgb8((s, m), rt.make_params(meta["width"], meta["height"], meta["spp"], meta["depth"],
                                                   meta["seed"]))
    path = str(tmp_path / "image.ppm")
    rt.save_ppm(path, img)
    mine = open(path, "rb").read()
    hdr = b"P6\n200 100\n255\n"
    assert ref[:len(hdr)] == hdr and mine[:len(hdr)] == hdr and len(mine) == len(ref)
    _u8_close(np.frombuffer(mine[len(hdr):], np.uint8), np.frombuffer(ref[len(hdr):], np.uint8))


# ---- caller streams that change between calls -----------------------------------
@pytest.mark.parametrize("streams,budget_samples", [(0, 4), (1, 4), (1, 0), (3, 0)])
def test_alternating_caller_streams(streams, budget_samples, opts):
    """One scene, renders alternating between two caller streams without host sync: the
    shared accumulation buffer (multi-pass frames), the workspaces (render_streams = 1) and the
    counters must never be used by both streams at once. Every frame equals its oracle."""
    torch = pytest.importorskip("torch")
    opts.set(render_streams=streams)
    W, H = 48, 32
    if budget_samples:
        opts.set(max_pass_bytes=W * H * 12 * budget_samples)
    s, m = G.scene("huge")
    ds = rt.DeviceScene((s, m))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = [(rt.make_params(W, H, 13, 64, k), O.camera_default(W, H, k % 2)) for k in range(6)]
    outs, segs = [], []
    for k, (p, cam) in enumerate(jobs):
        st = streams[k % 2]
        with torch.cuda.stream(st):
            outs.append(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"))
            segs.append(torch.zeros(3, dtype=torch.int64, device="cuda"))
        ds.render(cam, p, outs[-1].data_ptr(), st.cuda_stream, segs[-1].data_ptr())
    torch.cuda.synchronize()
    for k, (p, cam) in enumerate(jobs):
        want, want_seg = O.render_f32(s, m, cam, p)
        _bits_equal(outs[k].cpu().numpy(), want, f"frame {k}")
        assert int(segs[k][0]) == want_seg
    ds.close()


# ---- the wavefront variant (RT_FLAG_WAVEFRONT) -------------------------------
@pytest.mark.parametrize("queue_rays", [0, 1000])
def test_wavefront_variant_matches_megakernel(queue_rays, opts):
    """Per-segment launches through HBM ray queues (wave_gen_kernel, wave_bounce_kernel): the
    same frames, bit for bit, and the same segment counts as the persistent megakernel, on the
    huge scene (culled walk) and the simple scene (brute force, shading records in LDS), for
    depth limits 0..64, both cameras, and chunks smaller than a pass (wave_queue_rays)."""
    if queue_rays:
        opts.set(wave_queue_rays=queue_rays)
    for scene in ("huge", "simple"):
        s, m = G.scene(scene)
        for (W, H, spp, depth, mode) in [(64, 36, 4, 64, 0), (48, 27, 3, 64, 1), (40, 20, 5, 1, 0), (32, 16, 2, 0, 0),
                                         (33, 17, 9, 3, 1)]:
            cam = rt.Camera.default(W, H, mode)
            a, sa = rt.render_f32((s, m), rt.make_params(W, H, spp, depth, 7), cam)
            b, sb = rt.render_f32((s, m), rt.make_params(W, H, spp, depth, 7, wavefront=True), cam)
            _bits_equal(b, a, f"{scene} {W}x{H} spp {spp} depth {depth} camera {mode}")
            assert sb.segments == sa.segments and sb.primaries == sa.primaries


def test_wavefront_variant_golden_and_multipass(opts):
    """The wavefront variant against the reference's own frame (golden huge_64x36_s4) and a
    multi-pass render (slot budget of 8 samples) against the oracle."""
    meta, f32, _ = G.render("huge_64x36_s4")
    s, m = G.scene("huge")
    p = rt.make_params(meta["width"], meta["height"], meta["spp"], meta["depth"], meta["seed"], wavefront=True)
    img, _ = rt.render_f32((s, m), p)
    _bits_equal(img, f32, "golden huge_64x36_s4")
    W, H, spp = 40, 24, 21
    opts.set(max_pass_bytes=W * H * 12 * 8, wave_queue_rays=2000)
    cam = O.camera_default(W, H)
    img, st = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 3, wavefront=True), cam)
    want, want_seg = O.render_f32(s, m, cam, rt.make_params(W, H, spp, 64, 3))
    _bits_equal(img, want, "multi-pass")
    assert st.segments == want_seg


# ---- the deep-path split (RT_DEEP_SPLIT, render_kernel deep queue) --------------------------
@pytest.mark.parametrize("split", [1, 3, 8])
def test_deep_split_matches_unsplit(split, opts):
    """Paths that have traced deep_split segments move to the deep queue and finish in a second
    launch: the same frames, bit for bit, and the same segment counts as without the split
    (deep_split = 0), for both cameras, depth limits around the split, multi-pass frames (slot
    budget of 8 samples) and a deep queue that overflows (split 1 on 230 K samples with the
    corrected camera: 8 regions of 512 paths, most paths continue past their first segment),
    whose extra paths stay in the main launch. Configs 4 and 5 (test_full_config_frame_...) run
    with the default split, their passes being above deep_min_items."""
    opts.set(deep_min_items=0)  # split passes of any size
    s, m = G.scene("huge")
    cases = [(64, 36, 4, 64, 0, 0), (48, 27, 3, 64, 1, 0), (40, 20, 5, split, 0, 0),
             (33, 17, 9, split + 1, 1, 0), (40, 24, 21, 64, 0, 8), (160, 90, 16, 64, 1, 0)]
    for (W, H, spp, depth, mode, budget) in cases:
        cam = rt.Camera.default(W, H, mode)
        if budget:
            opts.set(max_pass_bytes=W * H * 12 * budget)
        opts.set(deep_split=0)
        a, sa = rt.render_f32((s, m), rt.make_params(W, H, spp, depth, 11), cam)
        opts.set(deep_split=split)
        b, sb = rt.render_f32((s, m), rt.make_params(W, H, spp, depth, 11), cam)
        opts.clear("max_pass_bytes")
        _bits_equal(b, a, f"split {split}: {W}x{H} spp {spp} depth {depth} camera {mode}")
        assert sb.segments == sa.segments and sb.primaries == sa.primaries


def test_deep_split_against_oracle_and_golden(opts):
    """With the split at 2 segments (most continuing paths go through the deep queue): the
    reference's own frame (golden huge_64x36_s4) and the oracle on a multi-pass render."""
    opts.set(deep_split=2, deep_min_items=0)
    meta, f32, _ = G.render("huge_64x36_s4")
    s, m = G.scene("huge")
    img, _ = rt.render_f32((s, m), rt.make_params(meta["width"], meta["height"], meta["spp"], meta["depth"],
                                                  meta["seed"]))
    _bits_equal(img, f32, "golden huge_64x36_s4")
    W, H, spp = 40, 24, 21
    opts.set(max_pass_bytes=W * H * 12 * 8)
    cam = O.camera_default(W, H, abi.RT_CAMERA_CORRECTED)
    img, st = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 5), rt.Camera.default(W, H, rt.CORRECTED))
    want, want_seg = O.render_f32(s, m, cam, rt.make_params(W, H, spp, 64, 5))
    _bits_equal(img, want, "multi-pass, corrected camera")
    assert st.segments == want_seg


def test_deep_split_overflow_feedback(opts):
    """One scene, frames with two cameras streamed without host sync, split at 1 segment on every
    pass: the corrected camera's passes overflow the deep queue, report it through host memory,
    and its later frames run unsplit, while the reference camera's frames keep the split. Every
    frame equals the unsplit render, bit for bit, with the same segment count."""
    torch = pytest.importorskip("torch")
    import time
    opts.set(deep_min_items=0, deep_split=1)
    W, H, spp = 160, 90, 16
    s, m = G.scene("huge")
    cams = [rt.Camera.default(W, H, rt.CORRECTED), rt.Camera.default(W, H)]
    ds = rt.DeviceScene((s, m))
    p = rt.make_params(W, H, spp, 64, 21)
    st = torch.cuda.current_stream()
    outs, segs = [], []
    for k in range(8):
        outs.append(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"))
        segs.append(torch.zeros(3, dtype=torch.int64, device="cuda"))
        ds.render(cams[k % 2].c, p, outs[-1].data_ptr(), st.cuda_stream, segs[-1].data_ptr())
        if k == 3:
            torch.cuda.synchronize()
            time.sleep(0.01)
    torch.cuda.synchronize()
    ds.close()
    opts.set(deep_split=0)
    for c, cam in enumerate(cams):
        want, want_st = rt.render_f32((s, m), p, cam)
        for k in range(c, 8, 2):
            _bits_equal(outs[k].cpu().numpy(), want, f"frame {k} camera {c}")
            assert int(segs[k][0]) == want_st.segments



def test_sample_pairs_through_the_deep_queue(opts):
    """Sample pairs whose samples leave for the deep queue: with the split at 1
    segment most continuing paths go there, so pairs end with one sample in each launch (the
    first's or the second's colour left in the pair slot) or with both queued (they meet through
    device-scope atomics, the second to end sums). Frames of different sizes and sample counts
    (pairs and single tail samples, several passes) follow each other on one scene, so every
    workspace's deep queue is laid out anew between passes (its pair-arrival words must start at
    zero). Every pass is planned as one issued beside other renders (diag in_flight: ring passes
    on the render streams, pairs taken every pass, not only when a render happens to be running;
    ADVICE r5), and the test checks that they were: rt_scene_usage.pair_passes for every frame,
    and, in the instrumented kernel, pair sums formed in the main launch and both-deep meets in
    the deep launch. Each frame equals the oracle bit for bit, as does the unpaired render."""
    torch = pytest.importorskip("torch")
    s, m = _glass_scene_frames()
    # one pass budget for the scene (8 samples of the largest frame): the frames below are cut
    # into passes of different sizes, single tail samples included
    opts.set(deep_min_items=0, deep_split=1, render_streams=0, max_pass_bytes=80 * 44 * 12 * 8, pairs=True,
             in_flight=True)
    cases = [(64, 40, 10), (48, 30, 23), (80, 44, 16), (40, 24, 7), (64, 40, 10), (80, 44, 26)]
    stream = torch.cuda.current_stream().cuda_stream
    for stats in (False, True):
        opts.set(stats=stats)
        ds = rt.DeviceScene((s, m))
        outs, splits = [], 0
        for W, H, spp in cases:
            o = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
            ds.render(rt.Camera.default(W, H), rt.make_params(W, H, spp, 64, 31), o.data_ptr(), stream)
            u = ds.usage()
            assert u["pair_passes"] >= 1, (W, H, spp, u)
            # (a camera whose deep queue overflowed is not split again for a while: the repeated
            # 64x40 and 80x44 frames may run unsplit)
            splits += u["split_passes"]
            outs.append(o)
        assert splits >= 4, splits  # the four first frames of their cameras at least
        torch.cuda.synchronize()
        if stats:
            ev = ds.debug_events()
            assert ev["pair_sums"] > 0 and ev["both_deep_meets"] > 0, ev
            ds.debug_counters()  # raises on a bounds-check violation
        ds.close()
        for (W, H, spp), o in zip(cases, outs):
            want, _ = O.render_f32(s, m, O.camera_default(W, H), rt.make_params(W, H, spp, 64, 31))
            _bits_equal(o.cpu().numpy(), want, f"{W}x{H} spp {spp} stats {stats}")
    opts.set(pairs=False, in_flight=False, stats=False)
    W, H, spp = cases[1]
    img, _ = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 31))
    want, _ = O.render_f32(s, m, O.camera_default(W, H), rt.make_params(W, H, spp, 64, 31))
    _bits_equal(img, want, "singles")


def _glass_scene_frames():
    """Small glass balls on the ground in front of the reference camera (rays trapped in them
    run to max_depth), a big glass sphere, lambert and metal balls."""
    rng = np.random.default_rng(5)
    n = 160
    s = np.zeros(n, dtype=abi.SPHERE_DTYPE)
    m = np.zeros(4, dtype=abi.MATERIAL_DTYPE)
    m[0] = (0, [0.5, 0.5, 0.5], 0.0)
    m[1] = (1, [0.7, 0.6, 0.5], 0.05)
    m[2] = (2, [1.0, 1.0, 1.0], 1.5)
    m[3] = (0, [0.8, 0.3, 0.2], 0.0)
    r = rng.choice([0.2, 0.3, 0.15], n).astype(np.float32)
    c = np.zeros((n, 3), dtype=np.float32)
    c[:, 0] = rng.uniform(-6, 6, n)
    c[:, 2] = rng.uniform(-6, 6, n)
    c[:, 1] = r
    s["center"], s["radius"], s["material"] = c, r, rng.choice([2, 2, 2, 0, 1, 3], n)
    s["center"][0], s["radius"][0], s["material"][0] = (0, -1000, 0), 1000.0, 0
    s["center"][1], s["radius"][1], s["material"][1] = (0, 1, 0), 1.0, 2
    return s, m


def test_lone_deep_launch_static_dealing_runs(opts):
    """The lone pass's deep launch (8-wave workgroups, shading records in LDS, chunks dealt
    statically from the regions' final counts) is taken when a split pass runs alone with the
    main launch's shading records in global memory, and reported by rt_scene_usage.deep_launch
    (8 | 16); frames in flight take the 4-wave launch (4). Both equal the unsplit render bit for
    bit, with the same segment counts (no test checked that the static path ran)."""
    torch = pytest.importorskip("torch")
    opts.set(deep_min_items=0, shade_global=True)
    s, m = G.scene("huge")
    W, H, spp = 640, 360, 64
    cam = rt.Camera.default(W, H)
    p = rt.make_params(W, H, spp, 64, 17)
    opts.set(deep_split=0)
    want, want_st = rt.render_f32((s, m), p, cam)
    opts.set(deep_split=8)
    ds = rt.DeviceScene((s, m))
    stream = torch.cuda.current_stream().cuda_stream
    outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(4)]
    segs = [torch.zeros(3, dtype=torch.int64, device="cuda") for _ in range(4)]
    ds.render(cam, p, outs[0].data_ptr(), stream, segs[0].data_ptr())
    torch.cuda.synchronize()
    lone = ds.usage()["deep_launch"]
    ds.close()
    # the in-flight plan, forced (diag in_flight) so that it does not depend on whether a render
    # is still running when the next call arrives
    opts.set(in_flight=True)
    ds = rt.DeviceScene((s, m))
    for o, g in zip(outs[1:], segs[1:]):
        ds.render(cam, p, o.data_ptr(), stream, g.data_ptr())
    flight = ds.usage()["deep_launch"]
    torch.cuda.synchronize()
    ds.close()
    assert lone == 8 | 16, lone
    assert flight == 4, flight
    for k, (o, g) in enumerate(zip(outs, segs)):
        _bits_equal(o.cpu().numpy(), want, f"frame {k}")
        assert int(g[0]) == want_st.segments


@pytest.mark.parametrize("streams", [0, 1])
def test_deep_split_variants_and_row_shares(streams, opts):
    """The split with the render variants (fast-math; brute force, the scalar-cache scene and the
    simple scene, which walk every sphere and are not split), on the caller's stream alone
    (render_streams = 1) or on the render streams, and for interleaved row shares: each equals its
    unsplit render."""
    opts.set(deep_min_items=0, render_streams=streams)
    W, H, spp = 72, 40, 8
    for scene, kw, rows in [("huge", dict(fast_math=True), {}), ("huge", dict(brute_force=True), {}),
                            ("huge", dict(scalar_scene=True), {}), ("simple", {}, {}),
                            ("huge", {}, dict(row_offset=2, row_stride=3, num_rows=13))]:
        s, m = G.scene(scene)
        cam = rt.Camera.default(W, H)
        p = rt.make_params(W, H, spp, 64, 9, **rows, **kw)
        opts.set(deep_split=0)
        a, sa = rt.render_f32((s, m), p, cam)
        opts.set(deep_split=2)
        b, sb = rt.render_f32((s, m), p, cam)
        _bits_equal(b, a, f"{scene} {kw} {rows}")
        assert sb.segments == sa.segments


def test_deep_split_streams_passes_of_changing_size(opts):
    """One DeviceScene, split passes of different pixel and sample counts streamed without host
    sync, so every workspace's deep-queue buffer serves passes of other sizes (its pixel flags
    must start cleared whatever the previous pass left there: rt_host.cpp deep_clean). Each
    frame equals its unsplit render, bit for bit, with the same segment count."""
    torch = pytest.importorskip("torch")
    opts.set(deep_min_items=0, deep_split=2)
    s, m = G.scene("huge")
    sizes = [(160, 90, 16), (48, 27, 3), (200, 120, 8), (64, 36, 4), (96, 54, 12), (40, 20, 5)] * 3
    ds = rt.DeviceScene((s, m))
    stream = torch.cuda.current_stream().cuda_stream
    outs, segs = [], []
    for k, (W, H, spp) in enumerate(sizes):
        outs.append(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"))
        segs.append(torch.zeros(3, dtype=torch.int64, device="cuda"))
        ds.render(rt.Camera.default(W, H, k % 2), rt.make_params(W, H, spp, 64, 30 + k), outs[-1].data_ptr(),
                  stream, segs[-1].data_ptr())
    torch.cuda.synchronize()
    ds.close()
    opts.set(deep_split=0)
    for k, (W, H, spp) in enumerate(sizes):
        want, st = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 30 + k), rt.Camera.default(W, H, k % 2))
        _bits_equal(outs[k].cpu().numpy(), want, f"frame {k} {W}x{H}@{spp}")
        assert int(segs[k][0]) == st.segments


# ---- the RCCL gather branch on one GPU (RT_DIAG_STANDIN_TRANSPORT) -------------------------
@pytest.mark.parametrize("n", [2, 8])
def test_multi_context_rccl_branch_with_standin_transport(n):
    """rt_multi_render_device's RCCL branch — grouped send/recv per peer on the ranks' own
    streams into slots of rank 0's gather buffer, then the de-interleave — with RCCL replaced by
    stream-ordered device copies between virtual ranks (the stand-in keeps RCCL's stream
    semantics: the receive waits for the sender's prior work, the sender's later work waits for
    the copy). Frames of different sizes (ragged tiles), formats, cameras and spp, enqueued back
    to back without host sync so that tiles and slots are reused while earlier frames are in
    flight, each equal to its single-device render; then the synchronous entry points."""
    torch = pytest.importorskip("torch")
    s, m = G.scene("huge")
    ctx = rt.MultiContext((s, m), devices=[0] * n, options=rt.options(standin_transport=True))
    assert ctx.n_ranks == n and ctx.uses_rccl
    jobs = [(48, 30, 8, 1, 0, False), (48, 30, 5, 2, 1, True), (64, 37, 12, 3, 0, False), (40, 9, 4, 4, 1, True),
            (48, 30, 6, 5, 0, True), (64, 37, 3, 6, 1, False)] * 2
    stream = torch.cuda.current_stream().cuda_stream
    outs = []
    for W, H, spp, seed, mode, u8 in jobs:
        outs.append(torch.empty((H, W, 3), dtype=torch.uint8 if u8 else torch.float32, device="cuda"))
        ctx.render_device(rt.Camera.default(W, H, mode), rt.make_params(W, H, spp, 64, seed), outs[-1].data_ptr(),
                          stream, rgb8=u8)
    torch.cuda.synchronize()
    for (W, H, spp, seed, mode, u8), o in zip(jobs, outs):
        p, cam = rt.make_params(W, H, spp, 64, seed), rt.Camera.default(W, H, mode)
        if u8:
            want, _ = rt.render_rgb8((s, m), p, cam)
            np.testing.assert_array_equal(o.cpu().numpy(), want)
        else:
            want, _ = rt.render_f32((s, m), p, cam)
            _bits_equal(o.cpu().numpy(), want, f"n={n} {W}x{H}@{spp}")
    p = rt.make_params(64, 37, 4, 64, 5)
    got, stm = ctx.render_f32(p)
    single, st1 = rt.render_f32((s, m), p)
    _bits_equal(got, single, "synchronous")
    assert stm.segments == st1.segments
    ctx.close()


# ---- a bounded HBM footprint (rt_options.max_workspace_bytes) ------------------------------
def test_workspace_cap_bounds_memory_with_the_same_bits(opts):
    """Under max_workspace_bytes the library takes one workspace per stream, then sample pairs
    (half the slot bytes), then smaller passes, then fewer streams: the scene's workspaces stay within the cap
    (rt_scene_usage_get), frames streamed without host sync keep the uncapped bits and segment
    counts, and a cap below one 4-sample pass is RT_ERR_CAPACITY."""
    torch = pytest.importorskip("torch")
    s, m = G.scene("huge")
    W, H, spp = 160, 90, 64
    cam = rt.Camera.default(W, H)
    p = rt.make_params(W, H, spp, 64, 17)
    want, want_st = rt.render_f32((s, m), p, cam)
    stream = torch.cuda.current_stream().cuda_stream
    per_sample = W * H * 12
    seen = set()
    for cap in (0, 64 << 20, 8 << 20, 4 << 20, 3 << 19):  # 1.5 MiB: one stream, 4-sample passes
        ds = rt.DeviceScene((s, m), options=rt.options(render_streams=7, max_workspace_bytes=cap))
        outs, segs = [], []
        for _ in range(4):
            outs.append(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"))
            segs.append(torch.zeros(3, dtype=torch.int64, device="cuda"))
            ds.render(cam, p, outs[-1].data_ptr(), stream, segs[-1].data_ptr())
        torch.cuda.synchronize()
        u = ds.usage()
        ds.close()
        for o, g in zip(outs, segs):
            _bits_equal(o.cpu().numpy(), want, f"cap {cap}")
            assert int(g[0]) == want_st.segments
        if cap:
            assert u["workspace_bytes"] <= cap, (cap, u)
        # a pass's slots: two sample pairs per full block of 4, one slot per tail sample
        ps = u["pass_samples"]
        assert u["workspace_bytes"] >= u["workspaces"] * (ps - 2 * (ps // 4)) * per_sample
        seen.add((u["render_streams"], u["workspaces"], u["pass_samples"]))
    assert len(seen) >= 3  # the caps changed the cut
    ds = rt.DeviceScene((s, m), options=rt.options(max_workspace_bytes=100 << 10))
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    with pytest.raises(rt.RtError) as e:
        ds.render(cam, p, out.data_ptr(), stream)
    assert e.value.status == abi.RT_ERR_CAPACITY
    ds.close()


# ---- ring passes (rt_options.ring_pass_bytes) -----------------------------------------------
def test_ring_passes_keep_the_bits_and_shrink_the_workspaces(opts):
    """With frames in flight, passes issued beside other renders hold at most ring_pass_bytes of
    slots (equal passes of a multiple of 4 samples, at least 32), while a frame issued alone runs
    whole in a workspace of its own: frames streamed without host sync keep the bits and segment
    counts of one-pass frames, the ring's workspaces hold the ring pass, and a ring size under 32
    samples leaves the passes as they were."""
    torch = pytest.importorskip("torch")
    s, m = G.scene("huge")
    W, H, spp = 160, 90, 96
    cam = rt.Camera.default(W, H)
    p = rt.make_params(W, H, spp, 64, 23)
    want, want_st = rt.render_f32((s, m), p, cam)
    stream = torch.cuda.current_stream().cuda_stream
    per_sample = W * H * 12
    for ring_samples, passes in ((40, 32), (64, 48), (28, None)):
        ds = rt.DeviceScene((s, m), options=rt.options(render_streams=3, ring_pass_bytes=per_sample * ring_samples))
        outs, segs = [], []
        for _ in range(5):
            outs.append(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"))
            segs.append(torch.zeros(3, dtype=torch.int64, device="cuda"))
            ds.render(cam, p, outs[-1].data_ptr(), stream, segs[-1].data_ptr())
        torch.cuda.synchronize()
        u = ds.usage()
        ds.close()
        for o, g in zip(outs, segs):
            _bits_equal(o.cpu().numpy(), want, f"ring passes of {ring_samples} samples")
            assert int(g[0]) == want_st.segments
        if passes is None:  # under 32 samples: no ring passes
            assert u["pass_samples"] == spp and u["workspaces"] == 6, u
        else:  # 96 samples in 3 (2) equal passes; 6 ring workspaces + the lone one
            assert u["pass_samples"] == passes and u["workspaces"] == 7, u
            assert u["workspace_bytes"] >= 6 * passes * per_sample + spp * per_sample


# ---- scenes at the LDS limit (the kernel's static LDS counts) --------------------
def test_scene_at_the_lds_limit_renders_or_is_refused():
    """A scene whose blob fits the device's LDS per workgroup only without the render kernel's
    static LDS (per-wave and per-lane arrays) must not reach a failing launch: brute force falls
    back to the scalar-cache kernel (the oracle's bits), the culled walk is refused with
    RT_ERR_UNSUPPORTED or renders correctly."""
    probe = rt.DeviceScene(G.scene("simple"))
    u = probe.usage()
    probe.close()
    assert 4096 < u["static_lds_bytes"] < 32768 and u["max_lds_bytes"] >= 65536
    # the brute-force blob is 20 B per geo slot (n_geo = pad4(n) + 4) + 32 B before the shading
    n_geo = ((u["max_lds_bytes"] - u["static_lds_bytes"] // 2 - 32) // 20) & ~3
    n = n_geo - 4
    rng = np.random.default_rng(3)
    s = np.zeros(n, dtype=abi.SPHERE_DTYPE)
    m = np.zeros(2, dtype=abi.MATERIAL_DTYPE)
    m[0] = (0, [0.5, 0.5, 0.5], 0.0)
    m[1] = (1, [0.7, 0.6, 0.5], 0.2)
    s["center"][:, 0] = rng.uniform(-30, 30, n)
    s["center"][:, 2] = rng.uniform(-30, 30, n)
    s["center"][:, 1] = 0.1
    s["radius"] = 0.1
    s["material"] = rng.integers(0, 2, n)
    s["center"][0], s["radius"][0] = (0, -1000, 0), 1000.0
    assert 20 * n_geo + 32 <= u["max_lds_bytes"] < 20 * n_geo + 32 + u["static_lds_bytes"]
    W, H, spp = 16, 8, 2
    cam = O.camera_default(W, H, abi.RT_CAMERA_CORRECTED)
    p = rt.make_params(W, H, spp, 8, 4)
    want, seg = O.render_f32(s, m, cam, p)
    got, st = rt.render_f32((s, m), rt.make_params(W, H, spp, 8, 4, brute_force=True), cam)
    _bits_equal(got, want, "brute force at the LDS limit")
    assert st.segments == seg
    try:
        got, st = rt.render_f32((s, m), p, cam)
    except rt.RtError as e:
        assert e.status == abi.RT_ERR_UNSUPPORTED, e
    else:
        _bits_equal(got, want, "culled at the LDS limit")


@pytest.mark.parametrize("spp,depth", [(1, 64), (2, 64), (5, 64), (7, 3), (13, 64), (6, 1)])
def test_sky_kernel_tail_samples(spp, depth, opts):
    """The sky kernel's blocked sum with tail samples (spp % 4 != 0: the reduce's tail after the
    blocks of 4, main.cxx:205) and without full blocks (spp < 4), at small depth limits: frames of
    the huge scene whose sky tiles it renders, lone (split) and back to back, equal the oracle's."""
    torch = pytest.importorskip("torch")
    opts.set(deep_min_items=0)
    s, m = G.scene("huge")
    W, H = 192, 96
    p = rt.make_params(W, H, spp, depth, 31)
    cam = rt.Camera.default(W, H)
    want, _ = O.render_f32(s, m, O.camera_default(W, H, 0), p)
    stream = torch.cuda.current_stream().cuda_stream
    ds = rt.DeviceScene((s, m))
    outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(3)]
    ds.render(cam, p, outs[0].data_ptr(), stream)
    torch.cuda.synchronize()
    sky = ds.usage()["sky_tiles"]
    for o in outs[1:]:
        ds.render(cam, p, o.data_ptr(), stream)
    torch.cuda.synchronize()
    ds.close()
    assert sky > 0
    for k, o in enumerate(outs):
        _bits_equal(o.cpu().numpy(), want, f"spp {spp} depth {depth} frame {k}")


@pytest.mark.parametrize("order", ["classes", "sky_serial", "no_sky", "natural_order"])
def test_dealing_orders_keep_the_bits(order, opts):
    """Passes dealt by tile classes (lead tiles first; the proven sky tiles by the
    sky kernel, beside the main launch or after it, or traced by the main launch), and in
    the natural order render the same bits as the oracle: a lone frame (split), frames in
    flight (split, ring passes), an interleaved row share, fast-math against its own natural
    order, and the corrected camera. rt_scene_usage reports the classes that were used."""
    torch = pytest.importorskip("torch")
    diag = {"classes": {}, "sky_serial": dict(sky_serial=True), "no_sky": dict(no_sky=True),
            "natural_order": dict(natural_order=True)}[order]
    opts.set(deep_min_items=0, **diag)
    s, m = G.scene("huge")
    stream = torch.cuda.current_stream().cuda_stream
    cases = [(320, 176, 12, {}, 0), (320, 176, 12, {}, 0), (256, 144, 8, dict(row_offset=3, row_stride=4, num_rows=36), 0),
             (192, 112, 8, {}, 1)]
    ds = rt.DeviceScene((s, m))
    outs, used = [], []
    for W, H, spp, rows, mode in cases:
        p = rt.make_params(W, H, spp, 64, 21, **rows)
        o = torch.empty((abi.rows_of(p), W, 3), dtype=torch.float32, device="cuda")
        ds.render(rt.Camera.default(W, H, mode), p, o.data_ptr(), stream)
        used.append(ds.usage())
        outs.append(o)
    torch.cuda.synchronize()
    ds.close()
    for (W, H, spp, rows, mode), o, u in zip(cases, outs, used):
        p = rt.make_params(W, H, spp, 64, 21, **rows)
        want, _ = O.render_f32(s, m, O.camera_default(W, H, mode), p)
        _bits_equal(o.cpu().numpy(), want, f"{order} {W}x{H} {rows} camera {mode}")
        if order == "natural_order":
            assert u["lead_tiles"] == 0 and u["sky_tiles"] == 0, u
        elif mode == 0:
            assert u["lead_tiles"] > 0, u
            assert (u["sky_tiles"] > 0) == (order in ("classes", "sky_serial")), u
    # the lone 320x176 frame is split (deep_min_items 0), in every order
    assert used[0]["split_passes"] == 1, used[0]
    # fast-math: the classes and the sky path change no bit of its own result either
    W, H, spp = 320, 176, 8
    p = rt.make_params(W, H, spp, 64, 5, fast_math=True)
    a, sa = rt.render_f32((s, m), p)
    opts.set(natural_order=True)
    b, sb = rt.render_f32((s, m), p)
    _bits_equal(a, b, f"fast-math {order} vs natural order")
    assert sa.segments == sb.segments
