"""bench.py's rank launch (CPU, gloo): `--gpus N` started without a launcher runs N ranks itself
(torch.distributed.run as a child process), and a WORLD_SIZE that disagrees with --gpus is an
error, never a silent one-GPU measurement (Missing #1 / Weak #5)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_bare_gpus2_launches_two_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                         timeout=240, env=_env(KGS_BENCH_BACKEND="gloo"), cwd="/tmp")
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line == {"n_gpus": 2, "ranks_joined": 2}


def test_world_size_must_match_gpus():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                         timeout=120, env=_env(WORLD_SIZE="1"), cwd="/tmp")
    assert out.returncode == 2
    assert "WORLD_SIZE=1" in out.stderr
    assert out.stdout.strip() == ""


def test_single_rank_default():
    out = subprocess.run([sys.executable, BENCH, "--launch-check"], capture_output=True, text=True, timeout=120,
                         env=_env(), cwd="/tmp")
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1]) == {"n_gpus": 1, "ranks_joined": 1}
