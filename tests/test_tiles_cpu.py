"""The dealing order of a pass (rt_tile_order): its 64-pixel blocks as a
permutation, lead tiles first, and the tiles proven to send every primary ray to the sky last.

The sky proof is what lets those samples skip the closest-hit test, so it is checked against
the reference's own closest hit (the CPU restatement, oracle_kat_hit = raytracer.hxx:94-118
brute force over every sphere): rays of every sky tile at the corners of its pixel range, with
the jitter at both ends of [0, 1), the lens offset at its extremes and at random points, built
in binary32 the way camera.hxx:46-57 builds them, must meet no sphere. Cameras: the reference's
(as shipped and corrected), row shares, and adversarial ones whose rays graze the ground and
the scene's spheres at the horizon. No GPU.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_binding as O
import raytracinginoneweekend_amd as rt
from raytracinginoneweekend_amd import _abi as abi

f32 = np.float32


def _rays(cam, W, H, xs, ys, us, vs, lens_dirs):
    """Primary rays (N, 6) as the kernel forms them in binary32 (main.cxx:192-200, camera.hxx:46-57)."""
    org = np.array(cam.origin, f32)
    llc, hor, ver = (np.array(v, f32) for v in (cam.lower_left_corner, cam.horizontal, cam.vertical))
    lens = f32(cam.lens_radius)
    out = []
    for x, y, U, V, r in zip(xs, ys, us, vs, lens_dirs):
        uu = f32(f32(x) / f32(W)) + f32(f32(U) / f32(W))
        vv = f32(f32(y) / f32(H)) + f32(f32(V) / f32(H))
        rd = np.array(r, f32) * lens
        off = np.array([uu * rd[0], vv * rd[1], f32(0)], f32)
        o = org + off
        d = ((llc + hor * uu) + ver * (f32(1) - vv)) - off
        if cam.mode == abi.RT_CAMERA_CORRECTED:
            d = d - org
        out.append(np.concatenate([o, d]).astype(f32))
    return np.array(out, f32)


def _hits(s, m, rays):
    n = len(rays)
    out = np.zeros(8 * n, np.uint32)
    O.lib().oracle_kat_hit(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s), abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m),
                           np.ascontiguousarray(rays).ctypes.data_as(C.POINTER(C.c_float)), n,
                           out.ctypes.data_as(C.POINTER(C.c_uint32)), None)
    return out.reshape(n, 8)[:, 0] != 0xffffffff


def _sky_rays(cam, W, H, row_offset, row_stride, perm, n_sky, rng, n_random=4):
    """Corner and random rays of every sky tile (8x8 tiles over the packed rows)."""
    tiles_x = W // 8
    top = 1.0 - 2.0 ** -24  # the largest jitter canonical() returns
    lens_dirs = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (.7071, .7071, 0), (-.7071, -.7071, 0)]
    xs, ys, us, vs, ls = [], [], [], [], []
    for b in perm[len(perm) - n_sky:]:
        ty, tx = divmod(int(b), tiles_x)
        x0, x1 = 8 * tx, 8 * tx + 7
        y0, y1 = row_offset + 8 * ty * row_stride, row_offset + (8 * ty + 7) * row_stride
        for x, U in ((x0, 0.0), (x1, top)):
            for y, V in ((y0, 0.0), (y1, top)):
                for r in lens_dirs:
                    xs.append(x); ys.append(y); us.append(U); vs.append(V); ls.append(r)
        for _ in range(n_random):
            v = rng.normal(size=3)
            v = v / np.linalg.norm(v) * rng.uniform() ** (1 / 3)
            xs.append(int(rng.integers(x0, x1 + 1))); ys.append(y0 + row_stride * int(rng.integers(0, 8)))
            us.append(float(rng.uniform(0, top))); vs.append(float(rng.uniform(0, top))); ls.append(tuple(v))
    return _rays(cam, W, H, xs, ys, us, vs, ls)


def _check(s, m, cam, W, H, row_offset=0, row_stride=1, num_rows=0, min_sky=1):
    p = rt.make_params(W, H, 4, 64, 1234, row_offset=row_offset, row_stride=row_stride, num_rows=num_rows)
    perm, n_lead, n_sky = rt.tile_order((s, m), p, cam)
    rows = num_rows or (H - row_offset + row_stride - 1) // row_stride
    assert len(perm) == W * rows // 64
    assert sorted(perm.tolist()) == list(range(len(perm)))  # a permutation of the blocks
    assert n_lead + n_sky <= len(perm)
    assert n_sky >= min_sky, (n_sky, len(perm))
    rays = _sky_rays(cam.c, W, H, row_offset, row_stride, perm, n_sky, np.random.default_rng(7))
    hit = _hits(s, m, rays)
    assert not hit.any(), f"{int(hit.sum())} rays of proven sky tiles meet a sphere"
    return perm, n_lead, n_sky


def test_reference_camera_config3_sky_tiles_meet_nothing():
    s, m = rt.huge_scene_arrays(1234)
    perm, n_lead, n_sky = _check(s, m, rt.Camera.default(1280, 720), 1280, 720, min_sky=10000)
    # the oracle's own classification (profiles/r06/deep_sources.txt): 10 567 tiles whose primaries
    # all reached the sky at 16 spp; the proof is conservative
    assert n_sky <= 10567 and n_lead >= 161


def test_row_shares_and_corrected_camera():
    s, m = rt.huge_scene_arrays(1234)
    for r, n in ((0, 8), (5, 8), (1, 2)):
        _check(s, m, rt.Camera.default(1280, 720), 1280, 720, row_offset=r, row_stride=n, min_sky=100)
    _check(s, m, rt.Camera.default(640, 360, rt.CORRECTED), 640, 360, min_sky=100)


@pytest.mark.parametrize("case", range(6))
def test_adversarial_cameras(case):
    """Cameras near the ground and among the spheres, looking at the horizon, up, and down: rays
    that graze the ground or pass just over a sphere must not be taken for sky."""
    s, m = rt.huge_scene_arrays(1234)
    rng = np.random.default_rng(100 + case)
    W, H = 320, 176
    pos = [(-4, 0.35, 5), (0, 0.05, 0), (6, 1.2, -3), (-11, 0.25, -11), (3, 2.5, 3), (0.5, 0.41, 0.7)][case]
    look = (float(rng.uniform(-8, 8)), float(rng.uniform(-0.5, 1.5)), float(rng.uniform(-8, 8)))
    cam = rt.Camera(pos, look, (0, 1, 0), W / H, float(rng.uniform(20, 90)), float(rng.uniform(0, 0.3)),
                    float(rng.uniform(0.5, 12)), rt.CORRECTED if case % 2 else rt.REFERENCE)
    _check(s, m, cam, W, H, min_sky=0)


def test_natural_order_without_whole_blocks():
    s, m = rt.huge_scene_arrays(1234)
    perm, n_lead, n_sky = rt.tile_order((s, m), rt.make_params(200, 100, 1), rt.Camera.default(200, 100))
    assert len(perm) == 0 and n_lead == 0 and n_sky == 0  # 20 000 pixels: not whole blocks of 64
