"""Loader for librt_mi355x.so (the HIP kernels + C-ABI built in-tree by csrc/Makefile).

There is no CPU fallback: if the library is missing or cannot load, every entry point
raises. torch (when installed) is imported first so that this library and torch share
one HIP runtime in the process (both resolve libamdhip64.so.7).
"""
import ctypes as C
import os

from . import _abi as abi

PKG = os.path.dirname(os.path.abspath(__file__))
# RT_LIB_PATH points at another build of the same C ABI (timing ablations only)
LIB_PATH = os.environ.get("RT_LIB_PATH") or os.path.join(PKG, "librt_mi355x.so")

_lib = None


class RtError(RuntimeError):
    """A failing C-ABI call: status code and rt_last_error() text."""

    def __init__(self, status, message):
        super().__init__(f"rt status {status}: {message}")
        self.status = status


def _declare(L):
    P = C.POINTER
    sig = {
        "rt_version": (C.c_int, []),
        "rt_last_error": (C.c_char_p, []),
        "rt_device_count": (C.c_int, [P(C.c_int)]),
        "rt_camera_init": (C.c_int, [P(C.c_float), P(C.c_float), P(C.c_float), C.c_float, C.c_float,
                                     C.c_float, C.c_float, C.c_uint32, P(abi.RtCamera)]),
        "rt_camera_default": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, P(abi.RtCamera)]),
        "rt_scene_simple": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(C.c_uint32), P(abi.RtMaterial),
                                      C.c_uint32, P(C.c_uint32)]),
        "rt_scene_huge": (C.c_int, [C.c_uint32, P(abi.RtSphere), C.c_uint32, P(C.c_uint32),
                                    P(abi.RtMaterial), C.c_uint32, P(C.c_uint32)]),
        "rt_scene_cuda": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(C.c_uint32), P(abi.RtMaterial),
                                    C.c_uint32, P(C.c_uint32)]),
        "rt_camera_cuda": (C.c_int, [C.c_uint32, C.c_uint32, P(abi.RtCamera)]),
        "rt_render_cuda_impl": (C.c_int, [C.c_uint32, C.c_uint32, P(C.c_uint8)]),
        "rt_release_cached": (C.c_int, []),
        "rt_tile_order": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32, P(abi.RtCamera),
                                    P(abi.RtParams), P(C.c_uint32), C.c_uint32, P(C.c_uint32), P(C.c_uint32),
                                    P(C.c_uint32)]),
        "rt_render_f32": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32,
                                    P(abi.RtCamera), P(abi.RtParams), P(C.c_float), P(abi.RtStats)]),
        "rt_render_rgb8": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32,
                                     P(abi.RtCamera), P(abi.RtParams), P(C.c_uint8), P(abi.RtStats)]),
        "rt_render_multi_f32": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32,
                                          P(abi.RtCamera), P(abi.RtParams), C.c_int, P(C.c_float),
                                          P(abi.RtStats)]),
        "rt_render_multi_rgb8": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32,
                                           P(abi.RtCamera), P(abi.RtParams), C.c_int, P(C.c_uint8),
                                           P(abi.RtStats)]),
        "rt_write_ppm": (C.c_int, [C.c_char_p, P(C.c_uint8), C.c_uint32, C.c_uint32]),
        "rt_multi_create": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32, P(C.c_int),
                                      C.c_int, P(C.c_void_p)]),
        "rt_multi_destroy": (C.c_int, [C.c_void_p]),
        "rt_multi_info": (C.c_int, [C.c_void_p, P(C.c_int), P(C.c_int)]),
        "rt_multi_render_device": (C.c_int, [C.c_void_p, P(abi.RtCamera), P(abi.RtParams), C.c_uint32, C.c_void_p,
                                             C.c_void_p]),
        "rt_multi_render_f32": (C.c_int, [C.c_void_p, P(abi.RtCamera), P(abi.RtParams), P(C.c_float),
                                          P(abi.RtStats)]),
        "rt_multi_render_rgb8": (C.c_int, [C.c_void_p, P(abi.RtCamera), P(abi.RtParams), P(C.c_uint8),
                                           P(abi.RtStats)]),
        "rt_scene_create": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32, C.c_int,
                                      P(C.c_void_p)]),
        "rt_scene_destroy": (C.c_int, [C.c_void_p]),
        "rt_render_device": (C.c_int, [C.c_void_p, P(abi.RtCamera), P(abi.RtParams), C.c_void_p, C.c_void_p,
                                       C.c_void_p]),
        "rt_scene_kernel_times": (C.c_int, [C.c_void_p, C.c_uint32, P(C.c_float), P(C.c_uint32)]),
        "rt_scene_debug_counters": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_int]),
        "rt_scene_debug_timeline": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_uint32, P(C.c_uint32)]),
        "rt_scene_debug_events": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_int]),
        "rt_epilogue_rgb8_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
        "rt_options_default": (C.c_int, [P(abi.RtOptions)]),
        "rt_options_parse": (C.c_int, [C.c_char_p, P(abi.RtOptions)]),
        "rt_set_default_options": (C.c_int, [P(abi.RtOptions)]),
        "rt_get_default_options": (C.c_int, [P(abi.RtOptions)]),
        "rt_scene_create_ex": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32, C.c_int,
                                         P(abi.RtOptions), P(C.c_void_p)]),
        "rt_scene_usage_get": (C.c_int, [C.c_void_p, P(abi.RtSceneUsage)]),
        "rt_multi_create_ex": (C.c_int, [P(abi.RtSphere), C.c_uint32, P(abi.RtMaterial), C.c_uint32, P(C.c_int),
                                         C.c_int, P(abi.RtOptions), P(C.c_void_p)]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("RT_LIB_PATH") and not hasattr(L, name):
            continue  # an older build under A/B may lack newer entry points
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return sig


EXPORTS = None


def lib():
    """The loaded C-ABI library (raises if it is not built)."""
    global _lib, EXPORTS
    if _lib is None:
        try:
            import torch  # noqa: F401  (share torch's HIP runtime when torch is present)
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RtError(-4, f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                              "or `make -C raytracinginoneweekend_amd/csrc`")
        L = C.CDLL(LIB_PATH)
        EXPORTS = _declare(L)
        _lib = L
    return _lib


def check(status):
    """Raise RtError for a non-zero C-ABI status."""
    if status != 0:
        raise RtError(status, lib().rt_last_error().decode(errors="replace"))
    return status
