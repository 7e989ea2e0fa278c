"""bench.py's multi-rank plumbing on the CPU: `bench.py --gpus N` started without a launcher
spawns N rank processes (torch.distributed.run, 127.0.0.1) before anything touches a GPU, and
the reported n_gpus is the world size; a WORLD_SIZE that disagrees with --gpus fails loudly.
--fake-device replaces the GPU work by no-op steps over gloo."""
import json
import os
import subprocess
import sys

import pytest

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_BENCH = os.path.join(_REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return env


def _last_json(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.parametrize("n", [1, 2])
def test_gpus_flag_spawns_world(n):
    r = subprocess.run([sys.executable, _BENCH, "--gpus", str(n), "--fake-device", "--steps", "3"],
                       capture_output=True, text=True, env=_env(), timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _last_json(r.stdout)
    assert rec["n_gpus"] == n
    assert rec["ranks"] == list(range(n))


def test_world_size_mismatch_fails():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, _BENCH, "--gpus", "2", "--fake-device", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stderr + r.stdout)
