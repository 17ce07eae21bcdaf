"""bench.py's multi-rank launcher (CPU): `--gpus N` without torchrun starts N
rank processes itself and reports the world size the process group saw; more
ranks than visible GPUs is refused before anything runs."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(*args, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("n", [1, 2])
def test_gpus_n_starts_n_ranks(n):
    r = _run("--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == n
    assert line["config"]["parallelism"] == f"dp{n}"
    assert line["config"]["global_batch"] == 4 * n
    assert line["steps"] == 3 and line["value"] > 0


def test_more_ranks_than_gpus_is_refused():
    import torch
    if torch.cuda.device_count() >= 64:
        pytest.skip("a machine with 64 GPUs")
    r = _run("--gpus", "64", "--steps", "1", "--warmup", "0")
    assert r.returncode != 0
    assert "visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], capture_output=True, text=True,
                       timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
