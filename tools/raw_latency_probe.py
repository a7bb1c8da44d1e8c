"""Per-call latency of the fused raw-line path vs line length, beside the
pre-normalized single-sentence path (spm_hip_encode_batch_host): where the
time of one Encode(line) call goes.  Usage: python tools/raw_latency_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sentencepiece-comments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import oracle_lib as O  # noqa: E402
import spm_amd as S  # noqa: E402


def timed(f, reps=400):
    for _ in range(20):
        f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    mb = open(os.path.join(ROOT, "tests", "golden", "test_model.model"), "rb").read()
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    base = b"The quick brown fox jumps over the lazy dog and keeps running. "
    for L in (0, 1, 25, 100, 200, 400, 800):
        line = (base * 20)[:L]
        raw_us = timed(lambda: dm.encode_raw_small([line]))
        norm = om.normalize([line])[0]
        buf, off = S.to_csr([norm])
        enc_us = timed(lambda: dm.encode_csr_host(buf, off))
        print("raw %4d B (norm %4d B): fused raw %7.1f us, encode only (normalized) %7.1f us"
              % (L, len(norm), raw_us, enc_us), flush=True)
    lines = open(os.path.join(ROOT, "tests", "golden", "botchan.txt"), "rb").read().split(b"\n")
    lines = [x for x in lines if x][:4288]
    for x in lines[:20]:
        dm.encode_raw_small([x])
    t0 = time.perf_counter()
    for x in lines:
        dm.encode_raw_small([x])
    dt = time.perf_counter() - t0
    ls = np.array([len(x) for x in lines])
    print("botchan %d lines (mean %.1f B, p50 %d, p90 %d, max %d): fused raw %.1f us/line"
          % (len(lines), ls.mean(), np.percentile(ls, 50), np.percentile(ls, 90), ls.max(), dt / len(lines) * 1e6),
          flush=True)
    for lo, hi in ((0, 40), (40, 80), (80, 120), (120, 10000)):
        sel = [x for x in lines if lo <= len(x) < hi][:300]
        if sel:
            t0 = time.perf_counter()
            for x in sel:
                dm.encode_raw_small([x])
            print("  %3d..%4d B: %d lines, %.1f us/line" % (lo, hi, len(sel), (time.perf_counter() - t0) / len(sel) * 1e6),
                  flush=True)
    dm.close()


if __name__ == "__main__":
    main()
