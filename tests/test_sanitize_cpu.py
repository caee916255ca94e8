"""CPU sanitizer runs (the reference has them commented out, CMakeLists.txt:105,123)
of the host-only half of the library (raytracinginoneweekend_amd/csrc/rt_host_build.cpp: the
reference's camera and scene constructors, the cluster and neighbour-list builder with its
walk-shortcut proofs, exact-division checks, options parser, PPM writer) and of the CPU
restatement (oracle/rt_oracle.cpp), built from the shipped sources by tests/sanitize/Makefile:

- AddressSanitizer + UndefinedBehaviorSanitizer (no recovery: the first report fails the run):
  tests/sanitize/host_check.cpp over every host entry point against the reference's fixtures,
  the restatement's render of every golden frame bit for bit, and the host-only tests of
  test_abi_cpu plus test_oracle_golden, test_iso_cpu and test_numerics_cpu with the sanitized
  libraries loaded into Python (LD_PRELOAD of libasan, RT_LIB_PATH / RT_ORACLE_SO);
- ThreadSanitizer: the restatement on 1 and 4 threads (the same bits) and the library's shared
  host state (exact-division cache, process-default options, thread-local errors) from 8 threads.
"""
import os
import subprocess
import sys

import pytest

import golden_io as G

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(REPO, "tests", "sanitize")
BUILD = os.path.join(SAN, "_build")


def _gcc_lib(name):
    out = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return out if os.path.isabs(out) and os.path.exists(out) else None


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-j4", "-C", SAN], check=True)
    return BUILD


def _run(cmd, env=None, timeout=600):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
             UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    e.update(env or {})
    r = subprocess.run(cmd, capture_output=True, text=True, env=e, timeout=timeout)
    report = [x for x in ("AddressSanitizer", "runtime error:", "ThreadSanitizer", "LeakSanitizer") if x in r.stderr]
    assert r.returncode == 0 and not report, f"{cmd[0]} rc={r.returncode} {report}\n{r.stderr[-4000:]}"
    return r


@pytest.mark.parametrize("exe", ["host_check_asan", "host_check_tsan"])
def test_host_half_sanitized(built, exe):
    r = _run([os.path.join(built, exe), "host", G.GOLDEN])
    assert "host_check host: ok" in r.stdout


def test_threads_under_tsan(built):
    _run([os.path.join(built, "host_check_tsan"), "threads", os.path.join(G.GOLDEN, "scene_huge_1234.bin")])


@pytest.mark.parametrize("name", sorted(n for n, m in G.manifest()["renders"].items() if m["rng"] == "pcg"))
def test_restatement_renders_goldens_under_asan(built, name):
    m = G.manifest()["renders"][name]
    scene = os.path.join(G.GOLDEN, G.manifest()["scenes"][m["scene"]]["file"])
    _run([os.path.join(built, "host_check_asan"), "render", scene, os.path.join(G.GOLDEN, m["f32"]),
          *(str(m[k]) for k in ("width", "height", "spp", "depth", "seed", "row_offset", "row_stride", "num_rows")),
          "1" if m["camera"] == "corrected" else "0", "4"])


def test_python_suites_with_sanitized_libraries(built):
    """test_oracle_golden, test_iso_cpu, test_numerics_cpu and the host-only tests of test_abi_cpu
    with the sanitized restatement and host half loaded into Python (leak checks off: the
    interpreter's own allocations are not ours)."""
    asan = _gcc_lib("libasan.so")
    if asan is None:
        pytest.skip("libasan.so not found next to g++")
    env = {"LD_PRELOAD": asan, "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
           "RT_ORACLE_SO": os.path.join(built, "librt_oracle_asan.so"),
           "RT_LIB_PATH": os.path.join(built, "librt_host_asan.so")}
    host_only = "generator or simple_scene or other_seeds or camera or capacity or ppm or cuda_variant or options"
    for args in (["tests/test_oracle_golden.py", "tests/test_iso_cpu.py", "tests/test_numerics_cpu.py"],
                 ["tests/test_abi_cpu.py", "-k", host_only]):
        r = _run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", *args], env=env, timeout=900)
        assert " passed" in r.stdout and " failed" not in r.stdout, r.stdout[-2000:]
