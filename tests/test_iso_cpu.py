"""The walk shortcut of dielectric spheres (rt_kernel.hip hint_candidate, rt_host.cpp
shortcut_words), checked as a geometric claim on the CPU with the reference's own binary32
arithmetic.

A lane whose last hit was a dielectric sphere S tests S first; when S has at most two neighbours
(the other clustered spheres whose AABB, grown by the walk's box pad for any origin in the ball,
meets the ball |p - C|^2 <= fl(fl(r r) 1.0201) plus a rounding margin) and both ends of the lane's
segment (0, fl(1.002 t_S)] lie in that ball, the kernel tests the neighbours and skips the cluster
walk. The claim: then no other clustered sphere's candidate (raytracer.hxx:52-91: near root in
(kMIN, kMAX), else far root) beats the minimum over S and its neighbours in the (t, index) order
of closest_hit (raytracer.hxx:94-118). Here rays start
on (and a few ulp off) the isolated spheres of the reference's huge scene, in every direction
including near-tangent ones, with |d| from 0.3 to 6; S's candidate and every other sphere's are
computed op by op in binary32, and every ray that passes the kernel's check is verified.
(The GPU tests check the kernel's bits with and without the shortcut.)"""
import numpy as np
import pytest

import golden_io as G

KMIN = np.float32(0.008)
GROW = np.float32(1.0201)  # rt_device.h kIsoR2Grow


def _cand(o, d, C, r):
    """The reference's candidate t of each (ray, sphere), inf when none; binary32 op by op."""
    f = np.float32
    ocx, ocy, ocz = (o[:, None, k] - C[None, :, k] for k in range(3))
    dx, dy, dz = (d[:, None, k] for k in range(3))
    a = (dx * dx + dy * dy) + dz * dz
    b = (ocx * dx + ocy * dy) + ocz * dz
    c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - (r * r)[None, :]
    disc = b * b - a * c
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        q = np.sqrt(np.where(disc > 0, disc, f(0)))
        t1 = (-b - q) / a
        t2 = (-b + q) / a
    fmax = np.float32(np.finfo(np.float32).max)
    ok1 = (disc > 0) & (t1 > KMIN) & (t1 < fmax)
    ok2 = (disc > 0) & ~ok1 & (t2 > KMIN) & (t2 < fmax)
    return np.where(ok1, t1, np.where(ok2, t2, np.float32(np.inf))).astype(np.float32)


def _fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def _neighbours(C, r, always, kinds, pad0):
    """rt_host.cpp shortcut_words, in double: {S: neighbours} for the spheres with a shortcut."""
    out = {}
    others = np.where(~always)[0]
    ra = np.abs(r.astype(np.float64))
    for S in np.where(kinds == 2)[0]:
        r2k = np.float32(np.float32(r[S] * r[S]) * GROW)
        rk = np.sqrt(np.float64(r2k))
        c1 = np.abs(C[S].astype(np.float64)).sum()
        R = rk * (1 + 1e-5) + 1e-5 * (c1 + 2 * rk) + 1e-30
        pad = 1e-3 * (c1 + 2 * R) + pad0 + 1e-6
        T = others[others != S]
        lo = C[T].astype(np.float64) - ra[T, None] - pad
        hi = C[T].astype(np.float64) + ra[T, None] + pad
        x = C[S].astype(np.float64)
        e = np.maximum(np.maximum(lo - x, 0.0), x - hi)
        nb = T[~((e * e).sum(1) > R * R * (1 + 1e-9))]
        if len(nb) <= 2:
            out[int(S)] = nb
    return out


def _scene(name):
    if name == "huge":
        return G.scene("huge")
    import test_gpu_parity as P  # the GPU tests' glass-ball scenes (touching and overlapping balls)
    seed, n, spread = {"glass_sparse": (7, 300, 12.0), "glass_dense": (7, 400, 6.0)}[name]
    return P._glass_scene(np.random.default_rng(seed), n, spread)


@pytest.mark.parametrize("name,min_short,min_nb", [("huge", 150, 30), ("glass_sparse", 150, 50),
                                                   ("glass_dense", 60, 40)])
def test_shortcut_claim(name, min_short, min_nb):
    s, m = _scene(name)
    C = np.ascontiguousarray(s["center"], dtype=np.float32)
    r = np.ascontiguousarray(s["radius"], dtype=np.float32)
    kinds = m["kind"][s["material"]]
    ra = np.abs(r)
    always = ra > 64 * np.median(ra)  # rt_host.cpp build_blob: the ground
    # the walk's box pad: at least the level-3 box's (the max over the scene's boxes)
    lo = (C - ra[:, None])[~always].min(0)
    hi = (C + ra[:, None])[~always].max(0)
    cc, ee = 0.5 * (lo + hi), 0.5 * (hi - lo)
    pad0 = 1e-3 * (np.abs(cc).sum() + ee.sum()) + 1e-6
    short = _neighbours(C, r, always, kinds, pad0)
    n_nb = sum(1 for v in short.values() if len(v))
    assert len(short) >= min_short and n_nb >= min_nb, (len(short), n_nb)
    others = np.where(~always)[0]
    rng = np.random.default_rng(2024)
    checked = 0
    for S, nb in short.items():
        n = 1000
        u = rng.normal(size=(n, 3))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        o = (C[S][None, :].astype(np.float64) + ra[S] * u).astype(np.float32)
        o = (o.view(np.int32) + rng.integers(-3, 4, size=o.shape).astype(np.int32)).view(np.float32)  # a few ulp off
        v = rng.normal(size=(n, 3))
        v /= np.linalg.norm(v, axis=1, keepdims=True)
        # a third near-tangent: the direction nearly in the tangent plane at o
        tang = v - (v * u).sum(1, keepdims=True) * u
        tang /= np.linalg.norm(tang, axis=1, keepdims=True)
        k = n // 3
        v[:k] = tang[:k] + rng.uniform(-1e-3, 1e-3, (k, 1)) * u[:k]
        d = (v * rng.uniform(0.3, 6.0, (n, 1))).astype(np.float32)
        tS = _cand(o, d, C[S:S + 1], r[S:S + 1])[:, 0]
        valid = np.isfinite(tS)
        # the kernel's check (hint_candidate): both ends of (0, fl(1.002 t)] in the ball
        oc = o - C[S][None, :]
        tq = (tS * np.float32(1.002)).astype(np.float32)
        q = _fma32(np.where(valid, tq, 0)[:, None], d, oc)
        o2 = (oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]
        q2 = (q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1]) + q[:, 2] * q[:, 2]
        r2k = np.float32(np.float32(r[S] * r[S]) * GROW)
        skip = valid & (o2 <= r2k) & (q2 <= r2k)
        if not skip.any():
            continue
        # the shortcut's minimum: S and its neighbours, in (t, index) order
        own = np.concatenate([[S], nb]).astype(np.int64)
        t_own = _cand(o[skip], d[skip], C[own], r[own])
        j = np.lexsort((np.broadcast_to(own, t_own.shape), t_own), axis=1)[:, 0]
        best_t = t_own[np.arange(len(j)), j]
        best_i = own[j]
        T = np.setdiff1d(others, own)
        tT = _cand(o[skip], d[skip], C[T], r[T])
        beats = (tT < best_t[:, None]) | ((tT == best_t[:, None]) & (T[None, :] < best_i[:, None]))
        assert not beats.any(), f"{name} sphere {S}: {int(beats.sum())} candidates beat the shortcut's minimum"
        checked += int(skip.sum())
    assert checked > 20000, checked
    print(f"{name}: {len(short)} glass spheres with a shortcut ({n_nb} with neighbours), rays checked {checked}")


@pytest.mark.parametrize("C,r", [((0.0, -1000.0, 0.0), 1000.0), ((1.5, 0.2, -3.0), 0.2), ((0.0, 1.0, 0.0), -0.95)])
def test_leaving_ray_gate_claim(C, r):
    """test_block8's gate for the always-tested spheres: a ray with b > 0 and c >= 0 (computed)
    and b 2^-22 < kMIN a has no candidate (raytracer.hxx:52-91) — checked op by op in binary32
    on rays from (and a few ulp around) the sphere's surface and from afar, near-tangent ones
    and ones with tiny |d| included."""
    rng = np.random.default_rng(7)
    Cf = np.array(C, dtype=np.float32)
    rf = np.float32(r)
    n = 400000
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    dist = np.where(rng.random(n) < 0.7, abs(r), abs(r) * rng.uniform(1.0, 3.0, n))
    o = (Cf.astype(np.float64) + dist[:, None] * u).astype(np.float32)
    o = (o.view(np.int32) + rng.integers(-4, 5, size=o.shape).astype(np.int32)).view(np.float32)
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    tang = v - (v * u).sum(1, keepdims=True) * u
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    k = n // 2
    v[:k] = tang[:k] + rng.uniform(-1e-4, 1e-2, (k, 1)) * u[:k]
    d = (v * np.exp(rng.uniform(np.log(1e-4), np.log(8.0), (n, 1)))).astype(np.float32)
    ocx, ocy, ocz = (o[:, j] - Cf[j] for j in range(3))
    dx, dy, dz = d[:, 0], d[:, 1], d[:, 2]
    a = (dx * dx + dy * dy) + dz * dz
    b = (ocx * dx + ocy * dy) + ocz * dz
    c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - rf * rf
    gate = (b > 0) & (c >= 0) & (b * np.float32(2.0 ** -22) < KMIN * a)
    assert gate.sum() > n // 10
    t = _cand(o[gate], d[gate], Cf[None, :], np.array([rf]))[:, 0]
    assert np.isinf(t).all(), f"{int(np.isfinite(t).sum())} gated rays have a candidate"
