"""The CPU restatement (oracle/) against fixtures produced by the reference itself.

This pins the oracle: every render and known-answer table below was computed by the
reference's own CPU path (oracle/_ref, tests/golden/make_golden.py), and the restatement
must reproduce it bit for bit before it is trusted to check the GPU.
"""
import ctypes as C

import numpy as np
import pytest

import golden_io as G
import oracle_binding as O
from raytracinginoneweekend_amd import _abi as abi

RENDERS = sorted(G.manifest()["renders"])


@pytest.mark.parametrize("name", RENDERS)
def test_render_bit_exact(name):
    meta, f32, u8 = G.render(name)
    s, m = G.scene(meta["scene"])
    cam = O.camera_default(meta["width"], meta["height"], G.camera_mode(meta))
    out, seg = O.render_f32(s, m, cam, G.params_for(meta), rng_mode=0 if meta["rng"] == "pcg" else 1)
    assert seg > 0
    np.testing.assert_array_equal(out.view(np.uint32), f32.view(np.uint32))
    np.testing.assert_array_equal(O.epilogue_rgb8(out), u8)


def test_camera_basis_matches_reference():
    meta, w = G.kat("camera", 0)
    n = meta["n"]
    basis = w[n * 9:].view(np.float32)
    cam = O.camera_default(meta["camera_w"], meta["camera_h"])
    mine = np.array(list(cam.origin) + list(cam.lower_left_corner) + list(cam.horizontal) +
                    list(cam.vertical) + [cam.lens_radius], dtype=np.float32)
    np.testing.assert_array_equal(mine.view(np.uint32), basis.view(np.uint32))


def test_kat_camera():
    meta, w = G.kat("camera", 9)
    n = meta["n"]
    rows = w[:n * 9].reshape(n, 9)
    cam = O.camera_default(meta["camera_w"], meta["camera_h"])
    inp = np.ascontiguousarray(rows[:, :3])
    out = np.zeros((n, 6), dtype=np.float32)
    O.lib().oracle_kat_camera(C.byref(cam), abi.ptr(inp, C.POINTER(C.c_uint32)), n,
                              abi.ptr(out, C.POINTER(C.c_float)))
    np.testing.assert_array_equal(out.view(np.uint32), rows[:, 3:])


def test_kat_hit_world():
    meta, w = G.kat("hit", 14)
    n = meta["n"]
    rows = w.reshape(n, 14)
    s, m = G.scene(meta["scene"])
    rays = np.ascontiguousarray(rows[:, :6]).view(np.float32)
    out = np.zeros((n, 8), dtype=np.uint32)
    O.lib().oracle_kat_hit(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s), abi.ptr(m, C.POINTER(abi.RtMaterial)),
                           len(m), abi.ptr(rays, C.POINTER(C.c_float)), n,
                           abi.ptr(out, C.POINTER(C.c_uint32)), None)
    assert (rows[:, 6] != 0xFFFFFFFF).sum() > n // 4  # the table exercises hits and misses
    np.testing.assert_array_equal(out, rows[:, 6:])


def test_kat_scatter():
    meta, w = G.kat("scatter", 23)
    n = meta["n"]
    rows = w.reshape(n, 23)
    _, m = G.scene(meta["scene"])
    inp = np.ascontiguousarray(rows[:, :11])
    out = np.zeros((n, 12), dtype=np.uint32)
    O.lib().oracle_kat_scatter(abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m), abi.ptr(inp, C.POINTER(C.c_uint32)),
                               n, abi.ptr(out, C.POINTER(C.c_uint32)))
    kinds = m["kind"][rows[:, 0]]
    assert set(np.unique(kinds)) == {0, 1, 2}
    assert (rows[:, 11] == 0).any() and (rows[:, 11] == 1).any()  # absorbed metal rays present
    np.testing.assert_array_equal(out, rows[:, 11:])


def test_kat_misc():
    meta, w = G.kat("misc", 28)
    n = meta["n"]
    rows = w.reshape(n, 28)
    inp = np.ascontiguousarray(rows[:, :12]).view(np.float32)
    out = np.zeros((n, 16), dtype=np.uint32)
    O.lib().oracle_kat_misc(abi.ptr(inp, C.POINTER(C.c_float)), n, abi.ptr(out, C.POINTER(C.c_uint32)))
    np.testing.assert_array_equal(out, rows[:, 12:])


def _fullframe():
    import json
    import os
    with open(os.path.join(G.GOLDEN, "fullframe.json")) as f:
        return json.load(f)


def test_fullframe_digests_cover_the_baseline_configs():
    """tests/golden/fullframe.json holds the reference's own whole-frame digests of BASELINE
    configs 2, 3, 4 and 5 (the GPU frame tests compare whole frames against every one of them,
    so a missing digest must fail here, not skip there): one 64-bit digest per row, every row
    present, at the BASELINE sizes."""
    ff = _fullframe()
    assert {"c2", "c3", "c4", "c5"} <= set(ff)
    sizes = {"c2": (1280, 720, 64, 50), "c3": (1280, 720, 128, 64), "c4": (3840, 2160, 256, 64),
             "c5": (1280, 720, 1024, 64)}
    for name, (W, H, spp, depth) in sizes.items():
        r = ff[name]
        assert (r["width"], r["height"], r["spp"], r["depth"]) == (W, H, spp, depth), name
    for name, r in ff.items():
        assert len(r["row_sha256_16"]) == r["height"] and len(r["sha256_f32"]) == 64
        assert r["seed"] == 1234 and r["camera"] == "reference" and r["rng"] == "pcg"


def test_restatement_reproduces_config2_whole_frame():
    """The restatement renders config 2 WHOLE (simple scene 1280x720 @64 spp, depth 50) with the
    same bits as the reference's own CPU path (sha256 of the f32 frame), and its per-row
    digests and channel sums agree."""
    import hashlib
    r = _fullframe()["c2"]
    W, H = r["width"], r["height"]
    s, m = G.scene("simple")
    out, _ = O.render_f32(s, m, O.camera_default(W, H), O.make_params(W, H, r["spp"], r["depth"], r["seed"]))
    assert hashlib.sha256(out.tobytes()).hexdigest() == r["sha256_f32"]
    np.testing.assert_allclose(out.astype(np.float64).sum(axis=(0, 1)), r["channel_sums"], rtol=0, atol=0)
    assert hashlib.sha256(O.epilogue_rgb8(out).tobytes()).hexdigest() == r["sha256_u8"]
