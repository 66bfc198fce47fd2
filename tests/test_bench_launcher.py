"""bench.py's multi-GPU launcher on CPU: `--gpus N` without
a launcher starts N rank processes itself (no exec, the parent never touches a
GPU), the ranks form one process group and rank 0 prints one JSON line with
n_gpus == N. `--dry-run` replaces the kernels with an empty timed step on gloo."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


def test_launcher_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    doc = json.loads(lines[0])
    assert doc["n_gpus"] == 2 and doc["ranks_seen"] == [0, 1] and doc["processes"] == 2
    assert doc["backend"] == "gloo"


def test_launcher_one_gpu_runs_in_process():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    doc = json.loads(r.stdout.strip().splitlines()[-1])
    assert doc["n_gpus"] == 1 and doc["processes"] == 1


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
