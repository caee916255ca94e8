"""TEST INFRASTRUCTURE: ctypes binding of the CPU restatement (oracle/_build/librt_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this. The
product package never imports it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from raytracinginoneweekend_amd import _abi as abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RT_ORACLE_SO: a sanitizer build of the same restatement (tests/test_sanitize_cpu.py)
ORACLE_SO = os.environ.get("RT_ORACLE_SO") or os.path.join(REPO, "oracle", "_build", "librt_oracle.so")
REF_DIR = os.path.join(REPO, "oracle", "_ref")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
        L = C.CDLL(ORACLE_SO)
        L.oracle_render_f32.restype = C.c_int
        L.oracle_render_f32.argtypes = [
            C.POINTER(abi.RtSphere), C.c_uint32, C.POINTER(abi.RtMaterial), C.c_uint32,
            C.POINTER(abi.RtCamera), C.POINTER(abi.RtParams), C.c_int, C.c_int,
            C.POINTER(C.c_float), C.POINTER(C.c_uint64)]
        L.oracle_render_cuda_compat.restype = C.c_int
        L.oracle_render_cuda_compat.argtypes = [
            C.POINTER(abi.RtSphere), C.c_uint32, C.POINTER(abi.RtMaterial), C.c_uint32,
            C.POINTER(abi.RtCamera), C.POINTER(abi.RtParams), C.c_int, C.POINTER(C.c_float),
            C.POINTER(C.c_uint64)]
        L.oracle_epilogue_rgb8.restype = None
        L.oracle_epilogue_rgb8.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.c_uint64]
        L.oracle_camera_init.restype = C.c_int
        L.oracle_camera_init.argtypes = [C.POINTER(C.c_float)] * 3 + [C.c_float] * 4 + [
            C.c_uint32, C.POINTER(abi.RtCamera)]
        L.oracle_camera_default.restype = C.c_int
        L.oracle_camera_default.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(abi.RtCamera)]
        L.oracle_kat_hit.restype = None
        L.oracle_kat_hit.argtypes = [C.POINTER(abi.RtSphere), C.c_uint32, C.POINTER(abi.RtMaterial),
                                     C.c_uint32, C.POINTER(C.c_float), C.c_uint32,
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
        L.oracle_kat_scatter.restype = None
        L.oracle_kat_scatter.argtypes = [C.POINTER(abi.RtMaterial), C.c_uint32, C.POINTER(C.c_uint32),
                                         C.c_uint32, C.POINTER(C.c_uint32)]
        L.oracle_kat_camera.restype = None
        L.oracle_kat_camera.argtypes = [C.POINTER(abi.RtCamera), C.POINTER(C.c_uint32), C.c_uint32,
                                        C.POINTER(C.c_float)]
        L.oracle_kat_misc.restype = None
        L.oracle_kat_misc.argtypes = [C.POINTER(C.c_float), C.c_uint32, C.POINTER(C.c_uint32)]
        _lib = L
    return _lib


def camera_default(width, height, mode=abi.RT_CAMERA_REFERENCE):
    cam = abi.RtCamera()
    assert lib().oracle_camera_default(width, height, mode, C.byref(cam)) == 0
    return cam


def make_params(width, height, spp, max_depth=64, seed=1234, row_offset=0, row_stride=1,
                num_rows=0, flags=0):
    return abi.RtParams(width, height, spp, max_depth, seed, row_offset, row_stride, num_rows, flags)


def render_f32(spheres, materials, camera, params, rng_mode=0, threads=None):
    """Linear RGB f32 image of shape (rows, width, 3) [or (height, width, 3) full frame]."""
    spheres = np.ascontiguousarray(spheres, dtype=abi.SPHERE_DTYPE)
    materials = np.ascontiguousarray(materials, dtype=abi.MATERIAL_DTYPE)
    rows = params.height if params.flags & abi.RT_FLAG_FULL_FRAME else abi.rows_of(params)
    out = np.zeros((rows, params.width, 3), dtype=np.float32)
    seg = C.c_uint64(0)
    threads = threads or min(8, os.cpu_count() or 1)
    rc = lib().oracle_render_f32(abi.ptr(spheres, C.POINTER(abi.RtSphere)), len(spheres),
                                 abi.ptr(materials, C.POINTER(abi.RtMaterial)), len(materials),
                                 C.byref(camera), C.byref(params), rng_mode, threads,
                                 abi.ptr(out, C.POINTER(C.c_float)), C.byref(seg))
    assert rc == 0, rc
    return out, seg.value


def render_cuda_compat(spheres, materials, camera, params, threads=None):
    """The reference CUDA variant's semantics (src/CUDA/cuda_impl.cu): f32 (rows, width, 3)."""
    spheres = np.ascontiguousarray(spheres, dtype=abi.SPHERE_DTYPE)
    materials = np.ascontiguousarray(materials, dtype=abi.MATERIAL_DTYPE)
    rows = params.height if params.flags & abi.RT_FLAG_FULL_FRAME else abi.rows_of(params)
    out = np.zeros((rows, params.width, 3), dtype=np.float32)
    seg = C.c_uint64(0)
    threads = threads or min(8, os.cpu_count() or 1)
    rc = lib().oracle_render_cuda_compat(abi.ptr(spheres, C.POINTER(abi.RtSphere)), len(spheres),
                                         abi.ptr(materials, C.POINTER(abi.RtMaterial)), len(materials),
                                         C.byref(camera), C.byref(params), threads,
                                         abi.ptr(out, C.POINTER(C.c_float)), C.byref(seg))
    assert rc == 0, rc
    return out, seg.value


def epilogue_rgb8(img):
    img = np.ascontiguousarray(img, dtype=np.float32)
    out = np.zeros(img.shape, dtype=np.uint8)
    lib().oracle_epilogue_rgb8(abi.ptr(img, C.POINTER(C.c_float)), abi.ptr(out, C.POINTER(C.c_uint8)),
                               img.size)
    return out
