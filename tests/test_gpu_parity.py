"""GPU parity: the HIP megakernel (through the C-ABI) against the reference's golden renders
and the CPU restatement (oracle/), bit for bit in f32.

Tolerance: the exact kernels are compiled with -ffp-contract=off and IEEE div/sqrt, so the
linear f32 framebuffer must match bitwise (0 ULP). The u8 epilogue evaluates powf through a
double pow; glibc's powf can differ in its last bit, so u8 may differ by 1 LSB on a handful
of texels (bound asserted below), never more.
"""
import numpy as np
import pytest

import golden_io as G
import oracle_binding as O
import raytracinginoneweekend_amd as rt
from raytracinginoneweekend_amd import _abi as abi

pytestmark = pytest.mark.gpu

RENDERS = sorted(n for n, m in G.manifest()["renders"].items() if m["rng"] == "pcg")
# clustered0: the same two-level walk with every cluster's members tested per lane (never
# transposed, rt_options.transpose_max = 0)
# ieee_roots: the IEEE sqrt/division sequences for the roots instead of their short exact forms
# (RT_DIAG_IEEE_ROOTS; rt_kernel.hip RayDiv)
VARIANTS = {"clustered": {}, "clustered0": {"_opts": {"transpose_max": 0}}, "brute": {"brute_force": True},
            "scalar": {"scalar_scene": True}, "ieee_roots": {"_opts": {"ieee_roots": True}}}


def _params(meta, **kw):
    return rt.make_params(meta["width"], meta["height"], meta["spp"], meta["depth"], meta["seed"],
                          meta["row_offset"], meta["row_stride"], meta["num_rows"], **kw)


def _bits_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    b = np.ascontiguousarray(b, dtype=np.float32).view(np.uint32)
    bad = np.count_nonzero(a != b)
    assert bad == 0, f"{bad} of {a.size} values differ; max |d| = " \
                     f"{np.max(np.abs(a.view(np.float32) - b.view(np.float32)))}"


@pytest.fixture(scope="module", autouse=True)
def _device():
    n = __import__("ctypes").c_int(0)
    rt.lib().rt_device_count(__import__("ctypes").byref(n))
    if n.value == 0:
        pytest.fail("no HIP device visible to librt_mi355x.so")


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("name", RENDERS)
def test_golden_render_f32(name, variant, opts):
    meta, f32, _ = G.render(name)
    scene = G.scene(meta["scene"])
    cam = rt.Camera.default(meta["width"], meta["height"], G.camera_mode(meta))
    kw = dict(VARIANTS[variant])
    opts.set(**kw.pop("_opts", {}))
    img, st = rt.render_f32(scene, _params(meta, **kw), cam)
    _bits_equal(img, f32)
    assert st.primaries == meta["width"] * meta["num_rows"] * meta["spp"]
    assert st.segments >= st.primaries


@pytest.mark.parametrize("name", RENDERS)
def test_golden_render_rgb8(name):
    meta, _, u8 = G.render(name)
    scene = G.scene(meta["scene"])
    cam = rt.Camera.default(meta["width"], meta["height"], G.camera_mode(meta))
    img, _ = rt.render_rgb8(scene, _params(meta), cam)
    diff = np.abs(img.astype(np.int16) - u8.astype(np.int16))
    assert diff.max() <= 1
    assert np.count_nonzero(diff) <= max(2, u8.size // 10000)


@pytest.mark.parametrize("scene_name,W,H,spp,depth,mode", [
    ("simple", 40, 24, 5, 64, abi.RT_CAMERA_REFERENCE),    # 1 block of 4 + 1 tail sample
    ("simple", 37, 19, 11, 50, abi.RT_CAMERA_CORRECTED),  # untiled width, 2 blocks + 3 tail
    ("huge", 64, 40, 8, 64, abi.RT_CAMERA_CORRECTED),
    ("huge", 24, 16, 3, 3, abi.RT_CAMERA_CORRECTED),     # shallow depth bound
    ("simple", 16, 8, 2, 1, abi.RT_CAMERA_REFERENCE),     # a single bounce
])
def test_against_oracle(scene_name, W, H, spp, depth, mode):
    s, m = G.scene(scene_name)
    cam = O.camera_default(W, H, mode)
    p = rt.make_params(W, H, spp, depth, 4321)
    ref, ref_seg = O.render_f32(s, m, cam, p)
    img, st = rt.render_f32((s, m), p, cam)
    _bits_equal(img, ref)
    assert st.segments == ref_seg  # same number of hit_world() calls: same paths


def test_max_depth_zero_is_black():
    s, m = G.scene("simple")
    img, st = rt.render_f32((s, m), rt.make_params(16, 8, 4, 0))
    assert not img.any() and st.segments == 0


def test_empty_scene_is_sky():
    s, m = G.scene("simple")
    p = rt.make_params(16, 8, 2, 64, 7)
    cam = O.camera_default(16, 8)
    ref, _ = O.render_f32(s[:0], m, cam, p)
    img, st = rt.render_f32((s[:0], m), p, cam)
    _bits_equal(img, ref)
    assert st.segments == st.primaries  # every primary misses


@pytest.mark.parametrize("W", [96, 128, 100])
def test_row_partition_invariance_full_frame(W):
    """Rows rendered by interleaved 'ranks' and stitched == one full render, bitwise, for widths
    in 8x8 tiles (96, 128: the tiled decomposition, with a ragged last tile row at H = 50) and
    not (100: row-major pixels)."""
    s, m = G.scene("huge")
    H, spp = 50, 4
    whole, _ = rt.render_f32((s, m), rt.make_params(W, H, spp, full_frame=True))
    cam = O.camera_default(W, H)
    for y in (0, 47, 48, 49):  # the tiled rows and the row-major remainder
        ref, _ = O.render_f32(s, m, cam, rt.make_params(W, H, spp, row_offset=y, num_rows=1))
        _bits_equal(whole[y:y + 1], ref)
    for n in (2, 3, 8, 16):
        acc = np.zeros_like(whole)
        for r in range(n):
            part, _ = rt.render_f32((s, m), rt.make_params(W, H, spp, row_offset=r, row_stride=n,
                                                           full_frame=True))
            acc[r::n] = part[r::n]
        _bits_equal(acc, whole)
    # packed (non full-frame) rows land in render order
    part, _ = rt.render_f32((s, m), rt.make_params(W, H, spp, row_offset=1, row_stride=3))
    _bits_equal(part, whole[1::3])


def test_config3_geometry_rows_match_oracle():
    """Full 1280x720 frame of the huge scene at low spp, checked on sampled rows."""
    s, m = G.scene("huge")
    W, H, spp = 1280, 720, 2
    img, st = rt.render_f32((s, m), rt.make_params(W, H, spp, full_frame=True))
    rows = [0, 97, 359, 360, 611, 719]
    cam = O.camera_default(W, H)
    for y in rows:
        ref, _ = O.render_f32(s, m, cam, rt.make_params(W, H, spp, row_offset=y, num_rows=1))
        _bits_equal(img[y:y + 1], ref)
    assert st.primaries == W * H * spp
    assert np.isfinite(img).all() and img.min() >= 0 and img.max() <= 1


def test_seed_changes_image():
    s, m = G.scene("simple")
    a, _ = rt.render_f32((s, m), rt.make_params(32, 16, 4, seed=1))
    b, _ = rt.render_f32((s, m), rt.make_params(32, 16, 4, seed=2))
    assert np.count_nonzero(a != b) > a.size // 4


def test_device_api_matches_host_api():
    torch = pytest.importorskip("torch")
    s, m = G.scene("huge")
    p = rt.make_params(128, 72, 4)
    host, _ = rt.render_f32((s, m), p)
    ds = rt.DeviceScene((s, m), device=0)
    out = torch.empty((72, 128, 3), dtype=torch.float32, device="cuda:0")
    seg = torch.zeros(3, dtype=torch.int64, device="cuda:0")
    stream = torch.cuda.current_stream()
    cam = rt.Camera.default(128, 72)
    for _ in range(2):  # workspace reuse across calls
        seg.zero_()
        ds.render(cam, p, out.data_ptr(), stream.cuda_stream, seg.data_ptr())
    torch.cuda.synchronize()
    _bits_equal(out.cpu().numpy(), host)
    assert int(seg[0].item()) > 128 * 72 * 4
    # without counters the non-counting instantiation renders: the same bits
    out.zero_()
    ds.render(cam, p, out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    _bits_equal(out.cpu().numpy(), host)
    u8 = torch.empty((72, 128, 3), dtype=torch.uint8, device="cuda:0")
    rt.epilogue_rgb8_device(out.data_ptr(), u8.data_ptr(), 128 * 72, stream.cuda_stream)
    torch.cuda.synchronize()
    ref8 = O.epilogue_rgb8(host)
    assert np.abs(u8.cpu().numpy().astype(int) - ref8.astype(int)).max() <= 1
    ds.close()


def _random_scene(rng, n, spread, center=(0.0, 0.0, 0.0)):
    """Adversarial scene: small spheres of mixed radii (some negative), exact duplicates with
    different materials (equal hit times in different clusters), a few big spheres."""
    s = np.zeros(n, dtype=abi.SPHERE_DTYPE)
    m = np.zeros(7, dtype=abi.MATERIAL_DTYPE)
    for i in range(7):
        m[i] = (i % 3, rng.uniform(0.2, 1.0, 3).astype(np.float32), [0.0, 0.3, 1.5][i % 3])
    c = (rng.uniform(-spread, spread, (n, 3)) + np.array(center)).astype(np.float32)
    c[:, 1] = np.abs(c[:, 1]) * 0.2 + center[1]
    r = rng.choice([0.05, 0.2, 0.3, 0.01], n).astype(np.float32)
    r[rng.random(n) < 0.05] *= -1
    s["center"], s["radius"], s["material"] = c, r, rng.integers(0, 7, n)
    dup = rng.choice(n, n // 10, replace=False)
    s["center"][dup[1::2]] = s["center"][dup[0::2][:len(dup[1::2])]]
    s["radius"][dup[1::2]] = s["radius"][dup[0::2][:len(dup[1::2])]]
    s["center"][0], s["radius"][0], s["material"][0] = (0, -1000.125, 0), 1000.0, 3
    s["center"][1], s["radius"][1], s["material"][1] = (center[0], 1 + center[1], center[2]), 1.0, 2
    return s, m


@pytest.mark.parametrize("seed,n,spread,center,mode", [
    (1, 600, 8.0, (0.0, 0.0, 0.0), abi.RT_CAMERA_CORRECTED),
    (2, 1500, 30.0, (0.0, 0.0, 0.0), abi.RT_CAMERA_REFERENCE),
    (3, 400, 3.0, (0.0, 0.0, 0.0), abi.RT_CAMERA_CORRECTED),
    (4, 800, 5.0, (200.0, 0.0, -150.0), abi.RT_CAMERA_CORRECTED),
    # a scene beyond 2^19 of the origin: the kernel keeps the IEEE root sequences
    (5, 300, 4.0, (7.0e5, 0.0, 0.0), abi.RT_CAMERA_CORRECTED),
])
@pytest.mark.parametrize("transpose", ["0", "4", "16"])
def test_cluster_culling_is_bit_exact(seed, n, spread, center, mode, transpose, opts):
    opts.set(transpose_max=int(transpose))
    rng = np.random.default_rng(seed)
    s, m = _random_scene(rng, n, spread, center)
    W, H, spp = 48, 32, 4
    cam = O.camera_default(W, H, mode)
    p = rt.make_params(W, H, spp, 64, seed)
    culled, st = rt.render_f32((s, m), p, cam)
    brute, sb = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, seed, brute_force=True), cam)
    _bits_equal(culled, brute)
    assert st.segments == sb.segments
    assert st.sphere_tests < sb.sphere_tests and st.box_tests > 0
    ref, seg = O.render_f32(s, m, cam, p)
    _bits_equal(culled, ref)
    assert st.segments == seg


def _glass_scene(rng, n, spread):
    """Small glass balls, the domain of the isolated-sphere shortcut (hint_candidate): isolated
    balls resting on the ground (as in the reference's huge scene), touching and overlapping
    neighbours, a ball with a bubble (negative radius) inside, exact duplicates, a big glass
    sphere, a few lambert/metal balls and the ground."""
    s = np.zeros(n, dtype=abi.SPHERE_DTYPE)
    m = np.zeros(5, dtype=abi.MATERIAL_DTYPE)
    m[0] = (0, [0.5, 0.5, 0.5], 0.0)
    m[1] = (1, [0.7, 0.6, 0.5], 0.1)
    m[2] = (2, [1.0, 1.0, 1.0], 1.5)
    m[3] = (2, [1.0, 1.0, 1.0], 1.33)
    m[4] = (0, [0.8, 0.3, 0.2], 0.0)
    r = rng.choice([0.2, 0.2, 0.2, 0.1, 0.35], n).astype(np.float32)
    c = np.zeros((n, 3), dtype=np.float32)
    c[:, 0] = rng.uniform(-spread, spread, n)
    c[:, 2] = rng.uniform(-spread, spread, n)
    c[:, 1] = r
    mat = rng.choice([2, 2, 3, 3, 2, 0, 1, 4], n)
    k = n // 8
    c[2:2 + k:2, 0] = c[3:3 + k:2, 0] + (r[2:2 + k:2] + r[3:3 + k:2])  # touching pairs (in float)
    c[2:2 + k:2, 2] = c[3:3 + k:2, 2]
    c[2 + k:2 + 2 * k:2, 0] = c[3 + k:3 + 2 * k:2, 0] + 0.5 * (r[2 + k:2 + 2 * k:2] + r[3 + k:3 + 2 * k:2])  # overlapping
    c[2 + k:2 + 2 * k:2, 2] = c[3 + k:3 + 2 * k:2, 2]
    c[5 * k], r[5 * k], mat[5 * k] = c[5 * k + 1], -0.8 * r[5 * k + 1], 2  # bubble in ball 5k + 1
    mat[5 * k + 1] = 2
    c[6 * k], r[6 * k] = c[6 * k + 1], r[6 * k + 1]                   # exact duplicate
    s["center"], s["radius"], s["material"] = c, r, mat
    s["center"][0], s["radius"][0], s["material"][0] = (0, -1000, 0), 1000.0, 0
    s["center"][1], s["radius"][1], s["material"][1] = (0, 1, 0), 1.0, 2
    return s, m


@pytest.mark.parametrize("seed,n,spread,mode,taken", [(7, 300, 12.0, abi.RT_CAMERA_REFERENCE, True),
                                                      (8, 500, 14.0, abi.RT_CAMERA_CORRECTED, True),
                                                      (9, 200, 8.0, abi.RT_CAMERA_CORRECTED, True),
                                                      (7, 400, 6.0, abi.RT_CAMERA_REFERENCE, False)])  # dense
def test_isolated_sphere_shortcut_is_bit_exact(seed, n, spread, mode, taken, opts):
    """Paths trapped in small glass balls skip the cluster walk when their segment stays inside
    an isolated ball (default on; RT_DIAG_NO_SHORTCUT off): the same bits as without the shortcut, as brute force
    and as the oracle, with the deep-path split at 3 segments (the deep launch takes the
    shortcut too); the instrumented kernel shows lanes taking it."""
    rng = np.random.default_rng(seed)
    s, m = _glass_scene(rng, n, spread)
    W, H, spp = 48, 32, 8
    cam = O.camera_default(W, H, mode)
    p = rt.make_params(W, H, spp, 64, seed)
    opts.set(deep_min_items=0, deep_split=3)
    on, st = rt.render_f32((s, m), p, cam)
    opts.set(no_shortcut=True)
    off, so = rt.render_f32((s, m), p, cam)
    opts.set(no_shortcut=False)
    _bits_equal(on, off)
    assert st.segments == so.segments
    assert st.box_tests <= so.box_tests
    if taken:
        assert st.box_tests < so.box_tests  # the shortcut was taken
    brute, sb = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, seed, brute_force=True), cam)
    _bits_equal(on, brute)
    ref, seg = O.render_f32(s, m, cam, p)
    _bits_equal(on, ref)
    assert st.segments == seg == sb.segments
    # the instrumented kernel: lanes took the shortcut, and whole iterations skipped the walk
    torch = pytest.importorskip("torch")
    ds = rt.DeviceScene((s, m), options=rt.options(rt.default_options(), stats=True))
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    ds.render(rt.Camera.default(W, H, mode), p, out.data_ptr(), stream)
    torch.cuda.synchronize()
    ev = ds.debug_events(reset=True)
    ds.close()
    _bits_equal(out.cpu().numpy(), ref)
    if taken:
        assert ev["iso_lanes"] > 0 and ev["walk_skipped"] > 0, ev


# ---- fast-math kernel: stated tolerance (SURVEY.md §8c "performance build") ---------------
# FMA-contracted discriminant, v_sqrt_f32 and reciprocal roots move hit times by a few ulp;
# a path whose hit/miss or reflect/refract decision flips diverges, so the bound is on the
# distribution, per pixel, on the linear f32 framebuffer:
#   >= 99% of pixels with max-channel |d| <= 1e-4, and mean |d| <= 1e-4 (spp >= 4);
#   u8 output within +-1 LSB on >= 99% of texels.
FAST_TOL_PIX, FAST_TOL_FRAC, FAST_TOL_MEAN = 1e-4, 0.99, 1e-4


@pytest.mark.parametrize("scene_name,W,H,spp,mode", [
    ("huge", 128, 72, 8, abi.RT_CAMERA_REFERENCE),
    ("huge", 96, 54, 4, abi.RT_CAMERA_CORRECTED),
    ("simple", 96, 48, 8, abi.RT_CAMERA_REFERENCE),
    ("simple", 64, 32, 4, abi.RT_CAMERA_CORRECTED),
])
def test_fast_math_within_stated_tolerance(scene_name, W, H, spp, mode):
    s, m = G.scene(scene_name)
    cam = O.camera_default(W, H, mode)
    p = rt.make_params(W, H, spp, 64, 99)
    ref, _ = O.render_f32(s, m, cam, p)
    img, st = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 99, fast_math=True), cam)
    d = np.abs(img - ref)
    frac = float((d.max(axis=-1) <= FAST_TOL_PIX).mean())
    assert frac >= FAST_TOL_FRAC, f"only {frac:.4%} of pixels within {FAST_TOL_PIX}"
    assert float(d.mean()) <= FAST_TOL_MEAN, f"mean |d| {d.mean():.3g}"
    assert np.isfinite(img).all()
    q = np.abs(O.epilogue_rgb8(img).astype(int) - O.epilogue_rgb8(ref).astype(int))
    assert (q <= 1).mean() >= 0.99


@pytest.mark.parametrize("ngpu", [0, 1, 2])
def test_render_multi_matches_single(ngpu):
    """rt_render_multi_f32 (row tiles over the visible devices, RCCL gather when N > 1) renders
    the same bits as one device. On a 1-GPU box every ngpu collapses to N = 1."""
    s, m = G.scene("huge")
    W, H, spp = 64, 37, 4  # H not divisible by 2: ragged tiles
    single, st1 = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 5))
    multi, stm = rt.render_multi_f32((s, m), rt.make_params(W, H, spp, 64, 5), ngpu=ngpu)
    _bits_equal(multi, single)
    assert stm.segments == st1.segments and stm.primaries == st1.primaries


@pytest.mark.parametrize("spp", [9, 16])
def test_multi_pass_slots_bit_exact(spp, opts):
    """A slot workspace smaller than the frame's slots forces several render passes whose
    partial sums are carried between passes; the addition order, hence the bits, must not
    change (config 5 at 1024 spp needs two passes)."""
    s, m = G.scene("huge")
    W, H = 64, 32
    one, st1 = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 3))
    opts.set(max_pass_bytes=W * H * 12 * 2)  # 2 slots per pass
    many, stn = rt.render_f32((s, m), rt.make_params(W, H, spp, 64, 3))
    _bits_equal(many, one)
    assert stn.segments == st1.segments


@pytest.mark.gpu
@pytest.mark.parametrize("budget_samples,shade", [(0, "shade_lds"), (0, "shade_global"), (0, ""), (4, ""),
                                                  (8, "shade_lds"), (12, "shade_global")])
def test_passes_and_shading_placement_bit_exact(budget_samples, shade, opts):
    """A small pass size (rt_options.max_pass_bytes) cuts the samples into passes of a multiple
    of 4, and the shading records may sit in LDS or global memory (RT_DIAG_SHADE_LDS /
    RT_DIAG_SHADE_GLOBAL); none of it may change the bits: the oracle's frame for spp = 23 (5
    blocks of 4 + a 3-sample tail)."""
    s, m = G.scene("huge")
    W, H, spp = 40, 24, 23
    p = rt.make_params(W, H, spp, 64, 11)
    cam = O.camera_default(W, H, abi.RT_CAMERA_REFERENCE)
    want, want_seg = O.render_f32(s, m, cam, p)
    if shade:
        opts.set(**{shade: True})
    if budget_samples:
        opts.set(max_pass_bytes=W * H * 12 * budget_samples)
    got, st = rt.render_f32((s, m), p)
    _bits_equal(got, want)
    assert st.segments == want_seg


@pytest.mark.gpu
@pytest.mark.parametrize("budget_samples,streams,ws", [
    (0, 2, 1), (4, 2, 1), (0, 3, 2), (4, 3, 2), (4, 4, 2), (0, 7, 2), (4, 8, 1), (4, 1, 2)])
def test_frames_in_flight_match_serial(budget_samples, streams, ws, opts):
    """Consecutive rt_render_device calls on one scene overlap (render passes on
    rt_options.render_streams internal streams with workspaces_per_stream workspaces each,
    partial grids while other renders run); every frame must still equal its serial render,
    with different cameras, spp and row partitions back to back and no sync between calls, in
    one pass per frame or in passes of 4 samples."""
    import torch
    opts.set(render_streams=streams, workspaces_per_stream=ws)
    if budget_samples:
        opts.set(max_pass_bytes=48 * 32 * 12 * budget_samples)
    s, m = G.scene("huge")
    W, H = 48, 32
    jobs = [(rt.make_params(W, H, 8, 64, 1), O.camera_default(W, H, abi.RT_CAMERA_REFERENCE), H),
            (rt.make_params(W, H, 5, 64, 2), O.camera_default(W, H, abi.RT_CAMERA_CORRECTED), H),
            (rt.make_params(W, H, 12, 64, 3, row_offset=1, row_stride=2), O.camera_default(W, H, 0), H // 2),
            (rt.make_params(W, H, 4, 7, 4), O.camera_default(W, H, abi.RT_CAMERA_CORRECTED), H)]
    ds = rt.DeviceScene((s, m))
    stream = torch.cuda.current_stream().cuda_stream
    outs, segs = [], []
    for p, cam, rows in jobs * 2:
        outs.append(torch.empty((rows, W, 3), dtype=torch.float32, device="cuda"))
        segs.append(torch.zeros(3, dtype=torch.int64, device="cuda"))
        ds.render(cam, p, outs[-1].data_ptr(), stream, segs[-1].data_ptr())
    torch.cuda.synchronize()
    for i, (p, cam, rows) in enumerate(jobs * 2):
        want, want_seg = O.render_f32(s, m, cam, p)
        _bits_equal(outs[i].cpu().numpy(), want)
        assert int(segs[i][0]) == want_seg
    ds.close()


# ---- the reference's CUDA variant (RT_FLAG_CUDA_COMPAT) ------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("scene_name,W,H,spp,depth,seed,rows", [
    ("cuda", 64, 36, 48, 32, 0, None), ("cuda", 50, 31, 7, 32, 5, None), ("cuda", 64, 36, 16, 3, 0, (1, 2)),
    ("cuda", 40, 30, 8, 0, 0, None), ("huge", 48, 32, 4, 32, 9, None), ("simple", 48, 27, 6, 64, 0, (0, 3))])
def test_cuda_compat_matches_oracle(scene_name, W, H, spp, depth, seed, rows):
    """compat_kernel (one lane per pixel, its xorshift32 engine sequential over the pixel's
    samples) against the CPU restatement of src/CUDA/cuda_impl.cu: bit-identical f32 frames
    and the same segment count, on the variant's scene and camera and on the CPU path's
    scenes, with row partitions. Parity with the variant itself is unpinned (no nvcc here)."""
    if scene_name == "cuda":
        s, m = rt.cuda_scene_arrays()
    else:
        s, m = G.scene(scene_name)
    kw = {} if rows is None else {"row_offset": rows[0], "row_stride": rows[1]}
    p = rt.make_params(W, H, spp, depth, seed, cuda_compat=True, **kw)
    cam = rt.Camera.cuda(W, H)
    got, st = rt.render_f32((s, m), p, cam)
    want, seg = O.render_cuda_compat(s, m, cam.c, p)
    _bits_equal(got, want)
    assert st.segments == seg


@pytest.mark.gpu
def test_cuda_impl_replacement_u8():
    """rt_render_cuda_impl(W, H, out) = cuda_impl(W, H, image_texels): the variant's scene,
    camera, 48 spp, 32 bounces, gamma 1/2.2 and (uint8)(255 c); +-1 LSB against the oracle's
    f32 frame through the CPU epilogue (powf rounding)."""
    W, H = 96, 54
    got = rt.render_cuda_impl(W, H)
    s, m = rt.cuda_scene_arrays()
    want, _ = O.render_cuda_compat(s, m, rt.Camera.cuda(W, H).c, rt.make_params(W, H, 48, 32, 0, cuda_compat=True))
    ref8 = O.epilogue_rgb8(want)
    assert np.abs(got.astype(int) - ref8.astype(int)).max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("cluster_size", [4, 8, 12, 24, 32, 64])
@pytest.mark.parametrize("transpose", [0, 16])
def test_cluster_size_bit_exact(cluster_size, transpose, opts):
    """Any cluster size (rt_options.cluster_size, read when the scene is created) gives the
    oracle's bits, with members tested per lane or transposed (clusters above 16 members always
    per lane)."""
    opts.set(cluster_size=cluster_size, transpose_max=transpose)
    rng = np.random.default_rng(11)
    for s, m in (G.scene("huge"), _random_scene(rng, 900, 10.0)):
        W, H, spp = 40, 24, 4
        cam = O.camera_default(W, H, abi.RT_CAMERA_CORRECTED)
        p = rt.make_params(W, H, spp, 64, 3)
        got, st = rt.render_f32((s, m), p, cam)
        want, seg = O.render_f32(s, m, cam, p)
        _bits_equal(got, want)
        assert st.segments == seg


@pytest.mark.gpu
@pytest.mark.parametrize("transpose", ["0", "16"])
def test_many_clusters_bit_exact(transpose, opts):
    """A scene with more than 128 clusters (5000 spheres) gives the oracle's bits."""
    opts.set(transpose_max=int(transpose))
    rng = np.random.default_rng(5)
    s, m = _random_scene(rng, 5000, 40.0)
    W, H, spp = 32, 24, 2
    cam = O.camera_default(W, H, abi.RT_CAMERA_CORRECTED)
    p = rt.make_params(W, H, spp, 64, 1)
    got, st = rt.render_f32((s, m), p, cam)
    want, seg = O.render_f32(s, m, cam, p)
    _bits_equal(got, want)
    assert st.segments == seg


@pytest.mark.gpu
@pytest.mark.parametrize("streams,W,H,spp,budget_samples", [(0, 96, 40, 9, 0), (1, 64, 33, 5, 0), (0, 50, 31, 7, 0),
                                                            (0, 96, 40, 8, 4), (1, 8, 8, 1, 0), (2, 200, 100, 3, 0),
                                                            (1, 96, 40, 8, 4)])
def test_guided_dealing_bit_exact(streams, W, H, spp, budget_samples, opts):
    """Guided dealing: each of the 8 queues owns 1/8 of the 64-item blocks and ticket t takes
    blocks [S(t), S(t+1)), chunks shrinking geometrically to 2 blocks (K = 12 for a pass issued
    alone, 6 beside other renders). Every item must be dealt exactly once: the oracle's bits and
    segment count, in one pass or several, on the caller's stream or the render streams, for
    tiny launches (one wave) and ragged sizes."""
    opts.set(render_streams=streams)
    if budget_samples:
        opts.set(max_pass_bytes=W * H * 12 * budget_samples)
    s, m = G.scene("huge")
    cam = O.camera_default(W, H, abi.RT_CAMERA_REFERENCE)
    p = rt.make_params(W, H, spp, 64, 21)
    got, st = rt.render_f32((s, m), p, cam)
    want, seg = O.render_f32(s, m, cam, p)
    _bits_equal(got, want)
    assert st.segments == seg
