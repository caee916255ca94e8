"""ctypes mirror of include/rt_api.h (the C-ABI boundary).

Record layouts are the C structs one for one; numpy dtypes are provided for the arrays
(spheres, materials) so scenes can be built and inspected without copies.
"""
import ctypes as C

import numpy as np

RT_OK = 0
RT_ERR_INVALID = -1
RT_ERR_DEVICE = -2
RT_ERR_CAPACITY = -3
RT_ERR_UNSUPPORTED = -4
RT_ERR_COMM = -5
RT_ERR_IO = -6

RT_OUTPUT_F32, RT_OUTPUT_RGB8 = 0, 1

RT_LAMBERT, RT_METAL, RT_DIELECTRIC = 0, 1, 2
RT_CAMERA_REFERENCE, RT_CAMERA_CORRECTED = 0, 1

RT_FLAG_FULL_FRAME = 1 << 0
RT_FLAG_FAST_MATH = 1 << 1
RT_FLAG_SCALAR_SCENE = 1 << 2
RT_FLAG_BRUTE_FORCE = 1 << 3
RT_FLAG_CUDA_COMPAT = 1 << 4  # semantics of src/CUDA/cuda_impl.cu
RT_FLAG_WAVEFRONT = 1 << 5  # A/B: per-segment launches with HBM ray queues (same bits)


class RtSphere(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("radius", C.c_float), ("material", C.c_uint32)]


class RtMaterial(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("albedo", C.c_float * 3), ("param", C.c_float)]


class RtCamera(C.Structure):
    _fields_ = [
        ("origin", C.c_float * 3),
        ("lower_left_corner", C.c_float * 3),
        ("horizontal", C.c_float * 3),
        ("vertical", C.c_float * 3),
        ("lens_radius", C.c_float),
        ("mode", C.c_uint32),
    ]


class RtParams(C.Structure):
    _fields_ = [
        ("width", C.c_uint32), ("height", C.c_uint32),
        ("spp", C.c_uint32), ("max_depth", C.c_uint32),
        ("seed", C.c_uint64),
        ("row_offset", C.c_uint32), ("row_stride", C.c_uint32), ("num_rows", C.c_uint32),
        ("flags", C.c_uint32),
    ]


class RtOptions(C.Structure):
    """rt_options (include/rt_api.h): resource bounds and same-bits variants of a scene."""
    _fields_ = [
        ("size", C.c_uint32), ("render_streams", C.c_uint32), ("workspaces_per_stream", C.c_uint32),
        ("deep_split", C.c_uint32), ("max_pass_bytes", C.c_uint64), ("max_workspace_bytes", C.c_uint64),
        ("deep_min_items", C.c_uint64), ("cluster_size", C.c_uint32), ("transpose_max", C.c_uint32),
        ("wave_queue_rays", C.c_uint32), ("diag", C.c_uint32), ("ring_pass_bytes", C.c_uint64),
    ]


class RtSceneUsage(C.Structure):
    _fields_ = [
        ("device_bytes", C.c_uint64), ("workspace_bytes", C.c_uint64), ("render_streams", C.c_uint32),
        ("workspaces", C.c_uint32), ("pass_samples", C.c_uint32), ("static_lds_bytes", C.c_uint32),
        ("max_lds_bytes", C.c_uint32), ("deep_launch", C.c_uint32), ("pair_passes", C.c_uint32),
        ("split_passes", C.c_uint32), ("lead_tiles", C.c_uint32), ("sky_tiles", C.c_uint32),
    ]


RT_DIAG = {
    "ieee_roots": 1 << 0, "no_shortcut": 1 << 1, "no_neighbours": 1 << 2, "no_root_box": 1 << 3,
    "shade_lds": 1 << 4, "shade_global": 1 << 5, "stats": 1 << 6, "stats_deep_only": 1 << 7, "verbose": 1 << 8,
    "standin_transport": 1 << 9, "unbounded_nb": 1 << 10, "no_pairs": 1 << 11, "pairs": 1 << 12,
    "in_flight": 1 << 13, "natural_order": 1 << 14, "no_sky": 1 << 15, "lone_unsplit": 1 << 16,
    "sky_serial": 1 << 17,
}


class RtStats(C.Structure):
    _fields_ = [
        ("primaries", C.c_uint64), ("segments", C.c_uint64), ("sphere_tests", C.c_uint64),
        ("box_tests", C.c_uint64),
        ("kernel_ms", C.c_double), ("wall_ms", C.c_double),
    ]


SPHERE_DTYPE = np.dtype([("center", "<f4", (3,)), ("radius", "<f4"), ("material", "<u4")])
MATERIAL_DTYPE = np.dtype([("kind", "<u4"), ("albedo", "<f4", (3,)), ("param", "<f4")])
assert SPHERE_DTYPE.itemsize == C.sizeof(RtSphere) == 20
assert MATERIAL_DTYPE.itemsize == C.sizeof(RtMaterial) == 20
assert C.sizeof(RtParams) == 40
assert C.sizeof(RtOptions) == 64 and C.sizeof(RtSceneUsage) == 56


def ptr(arr, ctype=C.c_void_p):
    """Pointer to a contiguous numpy array's data, typed for a ctypes argument."""
    assert arr.flags["C_CONTIGUOUS"]
    return C.cast(arr.ctypes.data, ctype)


def rows_of(params):
    """Number of rows a render covers (rt_params num_rows rule, include/rt_api.h)."""
    if params.num_rows:
        return params.num_rows
    st = params.row_stride or 1
    if params.row_offset >= params.height:
        return 0
    return (params.height - params.row_offset + st - 1) // st


def load_scene_file(path):
    """Scene fixture: 'RTSC' u32 version=1, u32 n_spheres, u32 n_materials, records."""
    raw = np.fromfile(path, dtype=np.uint8)
    hdr = raw[:16].view("<u4")
    if hdr[0] != 0x43535452 or hdr[1] != 1:
        raise ValueError(f"{path}: not an RTSC v1 scene file")
    ns, nm = int(hdr[2]), int(hdr[3])
    s = raw[16:16 + 20 * ns].view(SPHERE_DTYPE).copy()
    m = raw[16 + 20 * ns:16 + 20 * ns + 20 * nm].view(MATERIAL_DTYPE).copy()
    return s, m


def save_scene_file(path, spheres, materials):
    hdr = np.array([0x43535452, 1, len(spheres), len(materials)], dtype="<u4")
    with open(path, "wb") as f:
        f.write(hdr.tobytes())
        f.write(np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE).tobytes())
        f.write(np.ascontiguousarray(materials, dtype=MATERIAL_DTYPE).tobytes())
