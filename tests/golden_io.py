"""TEST INFRASTRUCTURE: loaders for the fixtures in tests/golden (see make_golden.py)."""
import json
import os

import numpy as np

from raytracinginoneweekend_amd import _abi as abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def scene(name):
    m = manifest()["scenes"][name]
    return abi.load_scene_file(os.path.join(GOLDEN, m["file"]))


def render(name):
    """(meta, f32 image (rows, W, 3), u8 image (rows, W, 3))."""
    m = manifest()["renders"][name]
    shape = (m["num_rows"], m["width"], 3)
    f32 = np.fromfile(os.path.join(GOLDEN, m["f32"]), dtype="<f4").reshape(shape)
    u8 = np.fromfile(os.path.join(GOLDEN, m["u8"]), dtype=np.uint8).reshape(shape)
    return m, f32, u8


def kat(name, ncols):
    m = manifest()["kats"][name]
    w = np.fromfile(os.path.join(GOLDEN, m["file"]), dtype="<u4")
    return m, w


def params_for(meta, flags=0):
    return abi.RtParams(meta["width"], meta["height"], meta["spp"], meta["depth"], meta["seed"],
                        meta["row_offset"], meta["row_stride"], meta["num_rows"], flags)


def camera_mode(meta):
    return abi.RT_CAMERA_CORRECTED if meta["camera"] == "corrected" else abi.RT_CAMERA_REFERENCE
