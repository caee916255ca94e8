"""Render entry points over the C-ABI (the replacement for `cuda_impl`, src/main.cxx:18,114).

render_f32 / render_rgb8   synchronous, host numpy buffers (rt_render_f32 / rt_render_rgb8)
DeviceScene.render         async on a caller stream into a device buffer (rt_render_device),
                           the path bench.py times with inputs resident in HBM
MultiContext               row tiles over ranks (devices), gathered to rank 0 (rt_multi_*)
save_ppm                   app::save_to_file (src/main.cxx:87-101), rt_write_ppm
"""
import contextlib
import ctypes as C
import os

import numpy as np

from . import _abi as abi
from ._lib import check, lib
from .camera import Camera


def make_params(width, height, spp, max_depth=64, seed=1234, row_offset=0, row_stride=1, num_rows=0,
                full_frame=False, scalar_scene=False, fast_math=False, brute_force=False, cuda_compat=False,
                wavefront=False):
    flags = (abi.RT_FLAG_FULL_FRAME if full_frame else 0) | (abi.RT_FLAG_SCALAR_SCENE if scalar_scene else 0) \
        | (abi.RT_FLAG_FAST_MATH if fast_math else 0) | (abi.RT_FLAG_BRUTE_FORCE if brute_force else 0) \
        | (abi.RT_FLAG_CUDA_COMPAT if cuda_compat else 0) | (abi.RT_FLAG_WAVEFRONT if wavefront else 0)
    return abi.RtParams(width, height, spp, max_depth, seed, row_offset, row_stride, num_rows, flags)


def options(base=None, **fields):
    """An rt_options record: the library defaults (or `base`) with `fields` set; diag bits by name
    (ieee_roots=True, stats=True, ...; include/rt_api.h rt_diag) or as diag=<int>."""
    o = abi.RtOptions()
    if base is None:
        check(lib().rt_options_default(C.byref(o)))
    else:
        C.memmove(C.byref(o), C.byref(base), C.sizeof(o))
    for k, v in fields.items():
        if k in abi.RT_DIAG:
            o.diag = (o.diag | abi.RT_DIAG[k]) if v else (o.diag & ~abi.RT_DIAG[k])
        elif k in dict(abi.RtOptions._fields_) and k != "size":
            setattr(o, k, int(v))
        else:
            raise KeyError(f"rt_options has no field {k!r}")
    return o


def parse_options(text, base=None):
    """rt_options_parse: "key=value,..." over `base` (default: the library defaults)."""
    o = options(base)
    check(lib().rt_options_parse(text.encode(), C.byref(o)))
    return o


def default_options():
    """The process default (rt_get_default_options): library defaults with RT_OPTIONS applied."""
    o = abi.RtOptions()
    check(lib().rt_get_default_options(C.byref(o)))
    return o


def set_default_options(opt=None):
    """rt_set_default_options (None: the library defaults)."""
    check(lib().rt_set_default_options(C.byref(opt) if opt is not None else None))


@contextlib.contextmanager
def default_options_set(**fields):
    """Within the block, scenes created without explicit options (the synchronous renders,
    DeviceScene(), MultiContext()) use the current defaults with `fields` changed."""
    prev = default_options()
    set_default_options(options(prev, **fields))
    try:
        yield
    finally:
        set_default_options(prev)


def _scene_arrays(scene):
    if isinstance(scene, tuple):
        s, m = scene
    else:
        s, m = scene.arrays()
    return (np.ascontiguousarray(s, dtype=abi.SPHERE_DTYPE), np.ascontiguousarray(m, dtype=abi.MATERIAL_DTYPE))


def _cam(camera, params):
    if camera is None:
        return Camera.default(params.width, params.height).c
    return camera.c if isinstance(camera, Camera) else camera


def _out_rows(params):
    return params.height if params.flags & abi.RT_FLAG_FULL_FRAME else abi.rows_of(params)


def render_f32(scene, params, camera=None):
    """Averaged linear RGB (before gamma) as float32 (rows, width, 3); returns (image, stats)."""
    s, m = _scene_arrays(scene)
    out = np.zeros((_out_rows(params), params.width, 3), dtype=np.float32)
    st = abi.RtStats()
    check(lib().rt_render_f32(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s), abi.ptr(m, C.POINTER(abi.RtMaterial)),
                              len(m), C.byref(_cam(camera, params)), C.byref(params),
                              abi.ptr(out, C.POINTER(C.c_float)), C.byref(st)))
    return out, st


def render_rgb8(scene, params, camera=None):
    """Gamma-corrected 8-bit RGB (rows, width, 3), as main.cxx:209-213 produces."""
    s, m = _scene_arrays(scene)
    out = np.zeros((_out_rows(params), params.width, 3), dtype=np.uint8)
    st = abi.RtStats()
    check(lib().rt_render_rgb8(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s), abi.ptr(m, C.POINTER(abi.RtMaterial)),
                               len(m), C.byref(_cam(camera, params)), C.byref(params),
                               abi.ptr(out, C.POINTER(C.c_uint8)), C.byref(st)))
    return out, st


def tile_order(scene, params, camera=None):
    """rt_tile_order: the pass's 64-pixel blocks in dealing order as
    (perm, n_lead, n_sky); perm is empty when the pass keeps the natural order."""
    s, m = _scene_arrays(scene)
    nb, nl, ns = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
    args = (abi.ptr(s, C.POINTER(abi.RtSphere)), len(s), abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m),
            C.byref(_cam(camera, params)), C.byref(params))
    check(lib().rt_tile_order(*args, None, 0, C.byref(nb), C.byref(nl), C.byref(ns)))
    perm = np.zeros(nb.value, dtype=np.uint32)
    if nb.value:
        check(lib().rt_tile_order(*args, abi.ptr(perm, C.POINTER(C.c_uint32)), nb.value, C.byref(nb), C.byref(nl),
                                  C.byref(ns)))
    return perm, nl.value, ns.value


def release_cached():
    """rt_release_cached: free the device context the synchronous renders keep between calls."""
    check(lib().rt_release_cached())


def render_multi_f32(scene, params, ngpu=0, camera=None):
    """Row-interleaved render over `ngpu` devices of this process, gathered with RCCL."""
    s, m = _scene_arrays(scene)
    out = np.zeros((params.height, params.width, 3), dtype=np.float32)
    st = abi.RtStats()
    check(lib().rt_render_multi_f32(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s),
                                    abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m), C.byref(_cam(camera, params)),
                                    C.byref(params), ngpu, abi.ptr(out, C.POINTER(C.c_float)), C.byref(st)))
    return out, st


def render_multi_rgb8(scene, params, ngpu=0, camera=None):
    """As render_multi_f32 with the gamma/u8 epilogue on every rank before the gather."""
    s, m = _scene_arrays(scene)
    out = np.zeros((params.height, params.width, 3), dtype=np.uint8)
    st = abi.RtStats()
    check(lib().rt_render_multi_rgb8(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s),
                                     abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m), C.byref(_cam(camera, params)),
                                     C.byref(params), ngpu, abi.ptr(out, C.POINTER(C.c_uint8)), C.byref(st)))
    return out, st


class MultiContext:
    """Persistent row-tile context over ranks (rt_multi_create): rank r renders rows r, r+N, ...
    on devices[r]; tiles are gathered to rank 0 (RCCL when every rank has its own device,
    device copies for ranks sharing rank 0's device) and de-interleaved into the frame."""

    def __init__(self, scene, devices=None, n_ranks=0, options=None):
        s, m = _scene_arrays(scene)
        h = C.c_void_p()
        devs = None
        if devices is not None:
            devs = (C.c_int * len(devices))(*devices)
            n_ranks = len(devices)
        check(lib().rt_multi_create_ex(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s),
                                       abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m), devs, n_ranks,
                                       C.byref(options) if options is not None else None, C.byref(h)))
        self.handle = h
        n, r = C.c_int(0), C.c_int(0)
        check(lib().rt_multi_info(h, C.byref(n), C.byref(r)))
        self.n_ranks, self.uses_rccl = n.value, bool(r.value)

    def render_f32(self, params, camera=None):
        out = np.zeros((params.height, params.width, 3), dtype=np.float32)
        st = abi.RtStats()
        check(lib().rt_multi_render_f32(self.handle, C.byref(_cam(camera, params)), C.byref(params),
                                        abi.ptr(out, C.POINTER(C.c_float)), C.byref(st)))
        return out, st

    def render_rgb8(self, params, camera=None):
        out = np.zeros((params.height, params.width, 3), dtype=np.uint8)
        st = abi.RtStats()
        check(lib().rt_multi_render_rgb8(self.handle, C.byref(_cam(camera, params)), C.byref(params),
                                         abi.ptr(out, C.POINTER(C.c_uint8)), C.byref(st)))
        return out, st

    def render_device(self, camera, params, d_out, stream=None, rgb8=False):
        """Enqueue a full frame into device pointer d_out on rank 0's device, `stream` order."""
        check(lib().rt_multi_render_device(self.handle, C.byref(_cam(camera, params)), C.byref(params),
                                           abi.RT_OUTPUT_RGB8 if rgb8 else abi.RT_OUTPUT_F32, C.c_void_p(d_out),
                                           C.c_void_p(stream or 0)))

    def close(self):
        if self.handle:
            lib().rt_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_cuda_impl(width, height):
    """cuda_impl(width, height, image_texels) (src/main.cxx:18, src/CUDA/cuda_impl.cu:384-453):
    the CUDA variant's scene, camera, 48 spp and 32 bounces; u8 RGB (height, width, 3)."""
    out = np.zeros((height, width, 3), dtype=np.uint8)
    check(lib().rt_render_cuda_impl(width, height, abi.ptr(out, C.POINTER(C.c_uint8))))
    return out


class DeviceScene:
    """A scene resident in HBM on one device (rt_scene_create); renders are stream-ordered."""

    def __init__(self, scene, device=0, options=None):
        s, m = _scene_arrays(scene)
        self.n_spheres, self.n_materials = len(s), len(m)
        h = C.c_void_p()
        check(lib().rt_scene_create_ex(abi.ptr(s, C.POINTER(abi.RtSphere)), len(s),
                                       abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m), device,
                                       C.byref(options) if options is not None else None, C.byref(h)))
        self.handle = h
        self.device = device

    def render(self, camera, params, d_rgb, stream=None, d_segments=None):
        """Enqueue a render into device pointer d_rgb (int address) on `stream` (int handle).
        d_segments: optional device int64[3] accumulating {segments, sphere tests, box tests}."""
        check(lib().rt_render_device(self.handle, C.byref(_cam(camera, params)), C.byref(params),
                                     C.c_void_p(d_rgb), C.c_void_p(stream or 0),
                                     C.c_void_p(d_segments) if d_segments else None))

    def usage(self):
        """rt_scene_usage_get: device bytes held and the last render's cut, as a dict."""
        u = abi.RtSceneUsage()
        check(lib().rt_scene_usage_get(self.handle, C.byref(u)))
        return {k: getattr(u, k) for k, _ in abi.RtSceneUsage._fields_}

    def kernel_times(self, max_calls=256):
        """Render-kernel durations (ms) of the most recent render() calls, oldest first."""
        buf = (C.c_float * max_calls)()
        n = C.c_uint32(0)
        check(lib().rt_scene_kernel_times(self.handle, max_calls, buf, C.byref(n)))
        return list(buf[:n.value])

    def debug_counters(self, reset=True):
        """Counters of the instrumented kernel (options stats=True), see rt_scene_debug_counters."""
        buf = (C.c_uint64 * 16)()
        check(lib().rt_scene_debug_counters(self.handle, buf, 1 if reset else 0))
        keys = ["wave_iters", "wave_refills", "wave_blocks", "lane_blocks", "wave_roots", "lane_roots", "segments",
                "wave_member_blocks", "cyc_refill", "cyc_start", "cyc_hit", "cyc_shade", "cyc_fold"]
        out = dict(zip(keys, list(buf)))
        out["items_dealt"] = buf[13]  # items (the deep launch: queued paths) the waves took
        out["launch_start"] = (~buf[14]) & 0xffffffffffffffff if buf[14] else 0  # 100 MHz ticks
        return out

    EVENTS = ["iter", "refill_trip", "fresh", "reject_trip", "lens_done", "scatter_done", "root_gate_pass", "super",
              "super_pass", "cluster_req", "transposed", "t_round", "t_far", "per_lane_members", "sky", "hit",
              "lambert", "unit_dir", "dielectric", "store", "metal_absorb", "live_lanes", "dry_iter", "dry_lanes",
              "iso_lanes", "walk_skipped", "walk_1", "walk_2", "walk_3_4", "walk_5_8", "pair_sums", "both_deep_meets"]

    def debug_events(self, reset=True):
        """Block-execution counts of the instrumented kernel (options stats=True), see rt_scene_debug_events."""
        buf = (C.c_uint64 * 32)()
        check(lib().rt_scene_debug_events(self.handle, buf, 1 if reset else 0))
        return dict(zip(self.EVENTS, list(buf)))

    def debug_timeline(self, max_waves=65536):
        """Per-wave (dry, exit, iterations, cu_id, refills, iterations_after_dry, start, cycles) of
        the last instrumented launch (options stats=True). For a deep launch two fields hold walk
        counts instead: dry = (walks with a walking lane that has no hint sphere) << 32 | walks,
        iterations_after_dry = iterations in which the wave walked the clusters. Otherwise dry =
        when the wave found every queue empty;
        times in ticks of the 100 MHz clock; cycles = shader-clock cycles in the loop, so
        cycles / (exit - start) x 100 MHz is the clock the wave ran at), see rt_scene_debug_timeline."""
        buf = (C.c_uint64 * (4 * max_waves))()
        n = C.c_uint32(0)
        check(lib().rt_scene_debug_timeline(self.handle, buf, max_waves, C.byref(n)))
        out = []
        for i in range(n.value):
            dry, ex, a, b = buf[4 * i], buf[4 * i + 1], buf[4 * i + 2], buf[4 * i + 3]
            start = (ex & ~0xffffffff) | (b & 0xffffffff)  # the start's low 32 bits, in the exit's epoch
            if start > ex:
                start -= 1 << 32
            out.append((dry, ex, a & 0xffff, b >> 48, (a >> 16) & 0xffff, (b >> 32) & 0xffff, start, a >> 32))
        return out

    def close(self):
        if self.handle:
            lib().rt_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def epilogue_rgb8_device(d_rgb, d_out, n_pixels, stream=None):
    check(lib().rt_epilogue_rgb8_device(C.c_void_p(d_rgb), C.c_void_p(d_out), n_pixels, C.c_void_p(stream or 0)))


def save_ppm(path, rgb8):
    """app::save_to_file (src/main.cxx:87-101) through rt_write_ppm: binary P6,
    'P6\\n<w> <h>\\n255\\n' then the (h, w, 3) texels."""
    rgb8 = np.ascontiguousarray(rgb8, dtype=np.uint8)
    h, w, _ = rgb8.shape
    check(lib().rt_write_ppm(os.fsencode(path), abi.ptr(rgb8, C.POINTER(C.c_uint8)), w, h))
