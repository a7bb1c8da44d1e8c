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


def test_compact_line_fits_the_driver_tail():
    """The printed line keeps every leg's numbers within ~6 KB (the driver's
    output tail keeps ~9 KB) and ends with the `legs` summary; the round-5
    full record (16 KB) is the input."""
    sys.path.insert(0, ROOT)
    import bench
    full = json.load(open(os.path.join(ROOT, "profiles", "r05f3_bench.json")))
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    text = json.dumps(line)
    assert len(text) <= 6000, len(text)
    assert list(line)[-1] == "legs"
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert {"c2", "c3", "ja", "c4", "c5", "bpe_train", "c1_line"} <= set(line["legs"])
    assert line["parity"]["mismatches_total"] == 0


def test_pmc_traffic_only_with_a_matching_stamp(tmp_path):
    """A PMC summary counts only when its source stamp equals the kernel
    sources the bench runs: a stale one gives traffic null and a note."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench
    import pmc_stamp
    good = {"hbm_bytes_per_launch": 1000.0, "src_sha": pmc_stamp.src_sha256()}
    json.dump(good, open(tmp_path / "legx__k_one.json", "w"))
    json.dump(dict(good, hbm_bytes_per_launch=500.0), open(tmp_path / "legx__k_two.json", "w"))
    t, info = bench.pmc_traffic(str(tmp_path), "legx", ["k_one", "k_two"])
    assert t == 1500.0 and len(info["traffic_source"]) == 2
    json.dump(dict(good, src_sha="0" * 64), open(tmp_path / "legx__k_two.json", "w"))
    t, info = bench.pmc_traffic(str(tmp_path), "legx", ["k_one", "k_two"])
    assert t is None and "stamped" in info["traffic_note"]
    t, info = bench.pmc_traffic(str(tmp_path), "legx", ["k_one", "k_three"])
    assert t is None and "no summary" in info["traffic_note"]


def test_pmc_traffic_encode_legs_drop_the_blocking_call(tmp_path):
    """Encode legs: the summary's last dispatch is bench.py's blocking call
    after the timed region (it also writes piece lengths), so the traffic is
    the mean of the other dispatches; the E-step keeps its own rule."""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench
    import pmc_stamp
    s = {"src_sha": pmc_stamp.src_sha256(), "hbm_bytes_per_launch": 1600.0,
         "read_bytes_per_dispatch": [800.0, 800.0, 800.0, 1000.0],
         "write_bytes_per_dispatch": [400.0, 400.0, 400.0, 1800.0]}
    json.dump(s, open(tmp_path / "c3__k.json", "w"))
    json.dump(s, open(tmp_path / "legx__k.json", "w"))
    assert bench.pmc_traffic(str(tmp_path), "c3", ["k"])[0] == 1200.0
    assert bench.pmc_traffic(str(tmp_path), "legx", ["k"])[0] == 1600.0
