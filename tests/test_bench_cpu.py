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


def test_parity_encode_periodic_reference_equals_direct():
    """bench.py's full-size encode check: for a corpus that repeats its first
    p sentences (the multi-byte leg), the oracle's output of those p, tiled,
    equals the oracle over the whole corpus; a changed token is counted."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    import oracle_lib as O
    gold = os.path.join(ROOT, "tests", "golden")
    mb = open(os.path.join(gold, "test_model.model"), "rb").read()
    om = O.OracleModel(mb)
    lines = [s for s in om.normalize(O.read_lines_binary(os.path.join(gold, "botchan.txt"))[:50])]
    reps = 7
    lens = np.tile(np.array([len(x) for x in lines], dtype=np.uint64), reps)[:50 * reps - 13]
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens, dtype=np.uint64)
    buf = np.frombuffer(b"".join(lines) * reps, dtype=np.uint8)[:int(off[-1])].copy()
    ids, plens, to = om.encode_normalized_csr(buf, off, threads=2, with_lens=True)
    r = bench.parity_encode(mb, buf, off, ids, plens, to, 2, period=50)
    assert r["mismatches"] == 0 and r["sentences"] == len(lens)
    ids2 = ids.copy()
    ids2[-1] += 1
    assert bench.parity_encode(mb, buf, off, ids2, plens, to, 2, period=50)["mismatches"] == 1
