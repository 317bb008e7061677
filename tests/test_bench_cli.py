"""bench.py's multi-rank launch (CPU, gloo): ``--gpus N`` without a torchrun environment must
start N ranks itself (one process each, as VSLURM:47's ``torchrun --nproc_per_node`` does) and
the gradient average they compute must be the rank mean -- the path the driver's N = 2/4/8
scaling runs take, here in ``--dry`` mode (stand-in gradient buffer, no GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, lines


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_launches_that_many_ranks(n):
    p, lines = _run("--gpus", str(n), "--dry", "--steps", "2", "--warmup", "1")
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1, p.stdout  # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["grad_avg_ok"] is True and out["ranks_ok"] == [True] * n


def test_single_rank_dry_run():
    p, lines = _run("--dry", "--steps", "1")
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(lines[-1])["n_gpus"] == 1
