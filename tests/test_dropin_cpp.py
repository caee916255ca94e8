"""The literal C++ drop-in (include/rt_render_impl.hpp) builds against the C ABI, fails with an
exception (as cuda_impl does) when no device is present, and on the GPU renders the same
bytes as the Python binding."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "raytracinginoneweekend_amd")


def _build(tmp_path):
    exe = str(tmp_path / "dropin")
    subprocess.run(["g++", "-std=c++20", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "examples", "dropin_main.cpp"), "-L", LIBDIR, "-lrt_mi355x",
                    f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_dropin_builds_and_reports_errors(tmp_path):
    exe = _build(tmp_path)
    import raytracinginoneweekend_amd as rt
    import ctypes
    n = ctypes.c_int(0)
    rt.lib().rt_device_count(ctypes.byref(n))
    if n.value:
        pytest.skip("device present: covered by the gpu test")
    r = subprocess.run([exe, str(tmp_path / "x.ppm")], capture_output=True, text=True)
    assert r.returncode == 3 and "render failed" in r.stderr


@pytest.mark.gpu
def test_dropin_matches_python_binding(tmp_path):
    exe = _build(tmp_path)
    out = tmp_path / "x.ppm"
    subprocess.run([exe, str(out), "4"], check=True)
    raw = out.read_bytes()
    hdr = b"P6\n200 100\n255\n"
    assert raw.startswith(hdr)
    img = np.frombuffer(raw[len(hdr):], dtype=np.uint8).reshape(100, 200, 3)
    import raytracinginoneweekend_amd as rt
    ref, _ = rt.render_rgb8(rt.simple_scene_arrays(), rt.make_params(200, 100, 4, 64, 1234))
    np.testing.assert_array_equal(img, ref)


@pytest.mark.gpu
def test_dropin_cuda_impl_matches_python_binding(tmp_path):
    """rt::cuda_impl (the CUDA variant's own shape and semantics) from C++ = rt.render_cuda_impl."""
    exe = _build(tmp_path)
    out = tmp_path / "c.ppm"
    subprocess.run([exe, str(out), "cuda"], check=True)
    raw = out.read_bytes()
    hdr = b"P6\n200 100\n255\n"
    assert raw.startswith(hdr)
    img = np.frombuffer(raw[len(hdr):], dtype=np.uint8).reshape(100, 200, 3)
    import raytracinginoneweekend_amd as rt
    np.testing.assert_array_equal(img, rt.render_cuda_impl(200, 100))
