"""bench.py's multi-process launcher on CPU (gloo): `--gpus N` outside
torchrun starts N ranks before any GPU call and rank 0 prints ONE line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run",
                        "--sentences", "1000"], capture_output=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    lines = [l for l in p.stdout.decode().splitlines() if l.strip()]
    assert len(lines) == 1, lines
    return json.loads(lines[0])


def test_bench_launcher_one_rank():
    line = _run(1)
    assert line["n_gpus"] == 1 and line["value"] == 1000.0


def test_bench_launcher_two_ranks():
    line = _run(2)
    assert line["n_gpus"] == 2 and line["value"] == 2000.0
    assert line["config"]["parallelism"] == "dp2"
