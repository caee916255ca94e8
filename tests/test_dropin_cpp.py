"""The C++ drop-in (include/rt_render_impl.hpp) against the reference's own output.

Two binaries:
* examples/_ref/ref_main_dropin — the REFERENCE's main() (src/main.cxx:104-118) with the
  INTEGRATION.md swap applied to a scratch copy and compiled against librt_mi355x.so by
  examples/build_ref_dropin.sh: its real raytracer::data / primitives::sphere /
  material::types / math::u8vec3, `rt::render_impl(raytracer_data, ...)` where `cuda_impl`
  was called (main.cxx:114), its own app::save_to_file. Built in its debug frame size
  (512x256, 16 spp). Its PPM must match the PPM the reference's CPU path writes for that frame
  (tests/golden/dropin_simple_512x256_s16.ppm) within 1 LSB.
* examples/dropin_main.cpp — a self-contained example with stand-in types; its 200x100 @1 spp
  PPM must match the reference-written config-1 PPM within 1 LSB.
Both fail like cuda_impl (an exception) when no device is present.
"""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "raytracinginoneweekend_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
REF_DROPIN = os.path.join(REPO, "examples", "_ref", "ref_main_dropin")


def _build(tmp_path):
    exe = str(tmp_path / "dropin")
    subprocess.run(["g++", "-std=c++20", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "examples", "dropin_main.cpp"), "-L", LIBDIR, "-lrt_mi355x",
                    f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def _has_device():
    import raytracinginoneweekend_amd as rt
    n = ctypes.c_int(0)
    rt.lib().rt_device_count(ctypes.byref(n))
    return n.value > 0


def _ppm(raw):
    """(header, texels) of a P6 file as app::save_to_file writes it (main.cxx:96-100)."""
    parts = raw.split(b"\n", 3)
    return b"\n".join(parts[:3]) + b"\n", np.frombuffer(parts[3], dtype=np.uint8)


def _u8_close(a, b):
    d = np.abs(a.astype(np.int16) - b.astype(np.int16))
    assert d.max() <= 1
    assert np.count_nonzero(d) <= max(2, a.size // 10000)


def test_dropin_builds_and_reports_errors(tmp_path):
    exe = _build(tmp_path)
    if _has_device():
        pytest.skip("device present: covered by the gpu test")
    r = subprocess.run([exe, str(tmp_path / "x.ppm")], capture_output=True, text=True)
    assert r.returncode == 3 and "render failed" in r.stderr


def test_reference_main_dropin_throws_without_device(tmp_path):
    """The reference's main() does not catch: like cuda_impl's check_errors (cuda_impl.cu:101-114)
    the drop-in throws std::runtime_error, which terminates the program."""
    if not os.path.exists(REF_DROPIN):
        pytest.skip("examples/_ref/ref_main_dropin not built (needs /root/reference: build())")
    if _has_device():
        pytest.skip("device present: covered by the gpu test")
    r = subprocess.run([REF_DROPIN], capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode != 0 and "rt_render_rgb8" in r.stderr


@pytest.mark.gpu
def test_reference_main_dropin_matches_reference_ppm(tmp_path):
    """The reference's own main() with cuda_impl swapped for rt::render_impl writes
    image_cuda.ppm (main.cxx:116); it equals the reference CPU path's PPM of the same frame
    (header byte for byte, texels within 1 LSB: device pow vs glibc powf), and its texels are
    exactly the library's u8 epilogue of a frame whose f32 bits are the reference's."""
    assert os.path.exists(REF_DROPIN), "examples/_ref/ref_main_dropin missing: run build() where the reference is"
    meta = json.load(open(os.path.join(GOLDEN, "dropin.json")))
    r = subprocess.run([REF_DROPIN], capture_output=True, text=True, cwd=tmp_path, timeout=120)
    assert r.returncode == 0, r.stderr
    hdr, mine = _ppm((tmp_path / "image_cuda.ppm").read_bytes())
    rhdr, ref = _ppm(open(os.path.join(GOLDEN, meta["ppm"]), "rb").read())
    assert hdr == rhdr == b"P6\n512 256\n255\n" and mine.size == ref.size == 512 * 256 * 3
    _u8_close(mine, ref)
    import hashlib
    import raytracinginoneweekend_amd as rt
    p = rt.make_params(meta["width"], meta["height"], meta["spp"], meta["depth"], meta["seed"])
    f32, _ = rt.render_f32(rt.simple_scene_arrays(), p)
    assert hashlib.sha256(f32.tobytes()).hexdigest() == meta["sha256_f32"]
    u8, _ = rt.render_rgb8(rt.simple_scene_arrays(), p)
    np.testing.assert_array_equal(mine, u8.reshape(-1))


@pytest.mark.gpu
def test_dropin_example_matches_reference_ppm(tmp_path):
    """examples/dropin_main.cpp at config 1 (200x100 @1 spp) against the PPM the reference's
    app::save_to_file wrote for that frame (tests/golden/c1_simple_200x100_s1.ppm)."""
    exe = _build(tmp_path)
    out = tmp_path / "x.ppm"
    subprocess.run([exe, str(out), "1"], check=True)
    hdr, mine = _ppm(out.read_bytes())
    rhdr, ref = _ppm(open(os.path.join(GOLDEN, "c1_simple_200x100_s1.ppm"), "rb").read())
    assert hdr == rhdr == b"P6\n200 100\n255\n"
    _u8_close(mine, ref)


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
