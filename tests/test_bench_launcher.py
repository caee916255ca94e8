"""bench.py's launcher on CPU: `python bench.py --gpus N` started as one process becomes the
launcher of N ranks (torch.distributed.run, rendezvous on 127.0.0.1) before anything touches a
GPU; with --launch-check every rank joins a gloo group, agrees on the world and exits without a
GPU call. The driver's own form (torch.distributed.run ... bench.py --gpus N) reaches the same
rank code directly."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lines(out):
    """Every JSON object in the ranks' merged stdout (lines of different ranks may interleave)."""
    dec, recs, i = json.JSONDecoder(), [], out.find("{")
    while i >= 0:
        obj, end = dec.raw_decode(out, i)
        if isinstance(obj, dict) and obj.get("launch_check"):
            recs.append(obj)
        i = out.find("{", end)
    return recs


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_ranks(n):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = _lines(r.stdout)
    assert sorted(x["rank"] for x in recs) == list(range(n))
    assert all(x["world"] == n and x["rank_sum"] == n * (n - 1) // 2 for x in recs)
    assert all(x["master_addr"] == "127.0.0.1" for x in recs)


def test_bench_single_rank_and_world_mismatch():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert _lines(r.stdout)[0]["world"] == 1
    env["WORLD_SIZE"] = "2"  # a launcher that started 2 ranks for --gpus 4 is refused
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
