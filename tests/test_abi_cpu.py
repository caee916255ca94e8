"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/rt_api.h
declares, and its host code (scene generator, camera basis, argument validation) matches
the reference. No compute call needs a GPU here.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import golden_io as G
import oracle_binding as O
import raytracinginoneweekend_amd as rt
from raytracinginoneweekend_amd import _abi as abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "rt_api.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = rt.lib()
    declared = _declared_symbols()
    assert len(declared) >= 14
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    from raytracinginoneweekend_amd import _lib
    assert set(declared) == set(_lib.EXPORTS), "ctypes declarations out of sync with rt_api.h"


def test_version():
    assert rt.lib().rt_version() == 2


def test_huge_scene_generator_matches_reference():
    s, m = rt.huge_scene_arrays(1234)
    gs, gm = G.scene("huge")
    assert len(s) == 486
    assert s.tobytes() == gs.tobytes() and m.tobytes() == gm.tobytes()
    # every index resolves (the reference's type-3 draws leave dangling indices otherwise)
    assert s["material"].max() < len(m)


def test_simple_scene_matches_reference():
    s, m = rt.simple_scene_arrays()
    gs, gm = G.scene("simple")
    assert s.tobytes() == gs.tobytes() and m.tobytes() == gm.tobytes()


@pytest.mark.parametrize("seed", [0, 1, 7, 99])
def test_huge_scene_other_seeds_well_formed(seed):
    s, m = rt.huge_scene_arrays(seed)
    assert 480 <= len(s) <= 490
    assert (s["radius"][5:] == np.float32(0.2)).all()
    assert s["material"].max() < len(m)
    assert set(np.unique(m["kind"])) <= {0, 1, 2}


@pytest.mark.parametrize("W,H,mode", [(200, 100, 0), (1280, 720, 0), (3840, 2160, 1), (37, 19, 1)])
def test_camera_basis_matches_oracle(W, H, mode):
    assert bytes(rt.Camera.default(W, H, mode).c) == bytes(O.camera_default(W, H, mode))


def test_camera_init_custom():
    cam = rt.Camera((1, 2, 3), (0, 0, -1), (0, 1, 0), 1.5, 60.0, 0.5, 2.0, rt.CORRECTED)
    ref = abi.RtCamera()
    f3 = C.c_float * 3
    O.lib().oracle_camera_init(f3(1, 2, 3), f3(0, 0, -1), f3(0, 1, 0), 1.5, 60.0, 0.5, 2.0, 1, C.byref(ref))
    assert bytes(cam.c) == bytes(ref)
    assert cam.basis()["lens_radius"] == 0.25


def test_invalid_arguments_fail_loudly():
    s, m = rt.simple_scene_arrays()
    with pytest.raises(rt.RtError) as e:
        rt.render_f32((s, m), rt.make_params(0, 10, 1))
    assert e.value.status == abi.RT_ERR_INVALID
    with pytest.raises(rt.RtError):
        rt.render_f32((s, m), rt.make_params(10, 10, 0))
    with pytest.raises(rt.RtError):  # rows past the bottom of the image
        rt.render_f32((s, m), rt.make_params(10, 10, 1, row_offset=5, num_rows=6))
    with pytest.raises(rt.RtError) as e:  # pixel index y W + x must fit 32 bits (sample keys)
        rt.render_f32((s, m), rt.make_params(1 << 16, 1 << 16, 1, num_rows=1))
    assert e.value.status == abi.RT_ERR_INVALID and "2^32" in str(e.value)
    bad = s.copy()
    bad["material"][0] = 99
    with pytest.raises(rt.RtError) as e:
        rt.DeviceScene((bad, m))
    assert "material index" in str(e.value)
    with pytest.raises(rt.RtError):
        rt.Camera.default(0, 10)


def test_scene_capacity_error():
    n = C.c_uint32(0)
    buf = np.zeros(2, dtype=abi.SPHERE_DTYPE)
    rc = rt.lib().rt_scene_simple(abi.ptr(buf, C.POINTER(abi.RtSphere)), 2, C.byref(n), None, 0, None)
    assert rc == abi.RT_ERR_CAPACITY and n.value == 5
    assert b"too small" in rt.lib().rt_last_error()


def test_raytracer_data_roundtrip():
    d = rt.RaytracerData()
    d.add_material(rt.Lambert((.1, .2, .5)))
    d.add_material(rt.Metal((.8, .6, .2), 0))
    d.add_material(rt.Dielectric(1, 1.5))
    d.add_material(rt.Lambert((.64, .8, .0)))
    d.add_sphere((0, 1, 0), 1.0, 0)
    d.add_sphere((0, -1000.125, 0), 1000.0, 3)
    d.add_sphere((2, 1, 0), 1.0, 1)
    d.add_sphere((-2, 1, 0), 1.0, 2)
    d.add_sphere((-2, 1, 0), -.99, 2)
    s, m = d.arrays()
    gs, gm = G.scene("simple")
    assert s.tobytes() == gs.tobytes() and m.tobytes() == gm.tobytes()


def test_save_ppm(tmp_path):
    img = np.arange(2 * 3 * 3, dtype=np.uint8).reshape(2, 3, 3)
    p = tmp_path / "x.ppm"
    rt.save_ppm(str(p), img)
    raw = p.read_bytes()
    assert raw.startswith(b"P6\n3 2\n255\n") and raw[len(b"P6\n3 2\n255\n"):] == img.tobytes()


def test_write_ppm_reproduces_reference_file(tmp_path):
    """rt_write_ppm on the reference's u8 frame of config 1 is byte for byte the file the
    reference's app::save_to_file wrote (tests/golden/c1_simple_200x100_s1.ppm)."""
    meta, _, u8 = G.render("c1_simple_200x100_s1")
    p = tmp_path / "image.ppm"
    rt.save_ppm(str(p), u8.reshape(meta["num_rows"], meta["width"], 3))
    assert p.read_bytes() == open(os.path.join(G.GOLDEN, meta["ppm"]), "rb").read()


def test_write_ppm_bad_path_fails_loudly(tmp_path):
    with pytest.raises(rt.RtError) as e:
        rt.save_ppm(str(tmp_path / "no" / "such" / "dir.ppm"), np.zeros((1, 1, 3), np.uint8))
    assert e.value.status == abi.RT_ERR_IO


# ---- the reference's CUDA variant (RT_FLAG_CUDA_COMPAT; src/CUDA/cuda_impl.cu) -------------
def test_cuda_variant_scene_and_camera():
    """rt_scene_cuda / rt_camera_cuda: cuda_impl.cu:425-437 and :371-375, the camera basis bit
    for bit as the oracle's camera ctor computes it for those arguments."""
    s, m = rt.cuda_scene_arrays()
    assert s["center"].tolist() == [[0, 0, -1], [0, -100.5, -1], [1, 0, -1], [-1, 0, -1], [-1, 0, -1]]
    assert s["radius"].tolist() == [np.float32(v) for v in (.5, 100., .5, .5, -.499)]
    assert s["material"].tolist() == [0, 3, 1, 2, 2]
    assert m["kind"].tolist() == [abi.RT_LAMBERT, abi.RT_METAL, abi.RT_DIELECTRIC, abi.RT_LAMBERT]
    assert m["param"].tolist() == [0, 0, 1.5, 0]
    cam = rt.Camera.cuda(1280, 720)
    f3 = C.c_float * 3
    want = abi.RtCamera()
    assert O.lib().oracle_camera_init(f3(0, 0, 0), f3(0, 0, -1), f3(0, 1, 0), np.float32(1280 / 720), 88.0, .0625,
                                      1.0, 0, C.byref(want)) == 0
    assert bytes(cam.c) == bytes(want)


def test_cuda_variant_oracle_engine_and_pixel_zero():
    """The restated xorshift32 engine (cuda_impl.cu:21-28) against the published sequence for
    state 1 (Marsaglia 2003: 270369, 67634689, 2647435461); and pixel 0 with seed 0, whose
    engine is the fixed point 0, renders (the default camera sends its rays to the sky)."""
    x, seq = 1, []
    for _ in range(3):
        x ^= (x << 13) & 0xffffffff
        x ^= x >> 17
        x ^= (x << 5) & 0xffffffff
        seq.append(x)
    assert seq == [270369, 67634689, 2647435461]
    s, m = rt.cuda_scene_arrays()
    W, H = 8, 6
    p = rt.make_params(W, H, 4, 32, 0, cuda_compat=True)
    img, seg = O.render_cuda_compat(s, m, rt.Camera.cuda(W, H).c, p)
    assert np.isfinite(img).all() and seg >= W * H * 4
    assert (img[0, 0] > 0).all()  # sky colour


def test_timed_kernel_code_hash():
    """bench.py stamps PMC summaries with the sha256 of the timed kernel's machine code and
    descriptor (rt::render_kernel<0, 7, false, false>), found in the library's gfx950 code object."""
    import bench
    h = bench.kernel_sha256()
    assert h is not None and len(h) == 64
    assert bench.kernel_sha256("no_such_kernel") is None


# ---- rt_options: the library's only tuning surface besides GPU_MAX_HW_QUEUES and RT_OPTIONS ----
def test_options_defaults_and_parse():
    o = rt.options()
    assert o.size == C.sizeof(abi.RtOptions)
    assert (o.render_streams, o.workspaces_per_stream, o.deep_split, o.max_pass_bytes, o.max_workspace_bytes,
            o.deep_min_items, o.cluster_size, o.transpose_max, o.wave_queue_rays, o.diag, o.ring_pass_bytes) == \
        (0, 2, 8, 2 << 30, 0, 1 << 25, 16, 16, 1 << 25, 0, 384 << 20)
    p = rt.parse_options("render_streams=3, max_workspace_bytes=0x100000000;deep_split=0 ieee_roots=1,stats=1,ring_pass_bytes=0")
    assert (p.render_streams, p.max_workspace_bytes, p.deep_split, p.ring_pass_bytes) == (3, 1 << 32, 0, 0)
    assert p.diag == abi.RT_DIAG["ieee_roots"] | abi.RT_DIAG["stats"]
    assert rt.parse_options("stats=0", p).diag == abi.RT_DIAG["ieee_roots"]
    assert rt.parse_options("").render_streams == 0  # empty text: unchanged


@pytest.mark.parametrize("text,field", [
    ("render_streams=9", "render_streams"), ("workspaces_per_stream=0", "workspaces_per_stream"),
    ("workspaces_per_stream=3", "workspaces_per_stream"), ("deep_split=2000", "deep_split"),
    ("max_pass_bytes=0", "max_pass_bytes"), ("max_pass_bytes=4294967296", "max_pass_bytes"),
    ("ring_pass_bytes=11", "ring_pass_bytes"), ("ring_pass_bytes=4294967296", "ring_pass_bytes"),
    ("cluster_size=6", "cluster_size"), ("cluster_size=68", "cluster_size"), ("transpose_max=17", "transpose_max"),
    ("wave_queue_rays=10", "wave_queue_rays"), ("diag=262144", "diag"), ("shade_lds=1,shade_global=1", "diag"),
    ("bogus=1", "bogus"), ("render_streams", "key=value"), ("render_streams=-1", "render_streams"),
    ("render_streams=x", "render_streams"), ("stats=2", "stats"), ("deep_split=4294967296", "deep_split")])
def test_options_rejected_with_the_field_named(text, field):
    base = rt.options()
    with pytest.raises(rt.RtError) as e:
        rt.parse_options(text, base)
    assert e.value.status == abi.RT_ERR_INVALID and field in str(e.value)
    assert base.render_streams == 0 and base.diag == 0  # the record is left as it was


def test_default_options_set_and_restore():
    before = rt.default_options()
    with rt.default_options_set(render_streams=5, no_shortcut=True):
        d = rt.default_options()
        assert d.render_streams == 5 and d.diag & abi.RT_DIAG["no_shortcut"]
    after = rt.default_options()
    assert bytes(after) == bytes(before)
    bad = rt.options()
    bad.size = 12
    with pytest.raises(rt.RtError) as e:
        rt.set_default_options(bad)
    assert "size" in str(e.value)


def test_rt_options_environment_applies_and_fails_loudly():
    """RT_OPTIONS is parsed once over the defaults; a malformed value makes every scene created
    without explicit options fail with the parser's message (never a silent default)."""
    import subprocess
    import sys
    code = ("import raytracinginoneweekend_amd as rt; o = rt.default_options(); "
            "print(o.render_streams, o.deep_split, o.max_workspace_bytes, o.diag)")
    env = dict(os.environ, RT_OPTIONS="render_streams=4,deep_split=0,max_workspace_bytes=4294967296,no_root_box=1")
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["4", "0", "4294967296", str(abi.RT_DIAG["no_root_box"])]
    env["RT_OPTIONS"] = "render_streams=40"
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True)
    assert out.returncode != 0 and "RT_OPTIONS" in out.stderr and "render_streams" in out.stderr


def test_multi_create_rejects_mixed_device_lists_before_any_device_call():
    """rt_multi_create accepts device lists that are all distinct (RCCL) or all rank 0's device
    (virtual ranks); a mix is RT_ERR_INVALID, decided before any HIP call (so also here, without a
    GPU), and the stand-in transport needs virtual ranks."""
    s, m = rt.simple_scene_arrays()
    for devs in ([0, 0, 1], [0, 1, 0], [1, 1, 2, 3]):
        with pytest.raises(rt.RtError) as e:
            rt.MultiContext((s, m), devices=devs)
        assert e.value.status == abi.RT_ERR_INVALID and "distinct" in str(e.value)
    with pytest.raises(rt.RtError) as e:
        rt.MultiContext((s, m), devices=[0, 1], options=rt.options(standin_transport=True))
    assert e.value.status == abi.RT_ERR_INVALID and "stand-in" in str(e.value)
