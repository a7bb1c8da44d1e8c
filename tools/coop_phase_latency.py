"""Phase cycles of the cooperative kernel for ONE sentence at a time (the
per-call latency case, no other waves on the GPU): each call encodes one
botchan line (60..120 normalized bytes, test_model.model) through the
small-call path (coop_small_kernel).  Run with SPM_HIP_COOP_PROF=1; the per-call phase lines go to
stderr.  Usage: SPM_HIP_COOP_PROF=1 python tools/coop_phase_latency.py 2> prof.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sentencepiece-comments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
import spm_amd as S  # noqa: E402


def main():
    mb = open(os.path.join(ROOT, "tests", "golden", "test_model.model"), "rb").read()
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    lines = [x for x in open(os.path.join(ROOT, "tests", "golden", "botchan.txt"), "rb").read().split(b"\n") if x]
    norm = [x for x in om.normalize(lines[:600]) if 60 <= len(x) <= 120][:300]
    tiny = []
    for x in norm:
        buf, off = S.to_csr([x] + tiny)
        dm.encode_csr_host(buf, off)
    print("sentences", len(norm), "mean bytes", sum(map(len, norm)) / len(norm), flush=True)
    dm.close()


if __name__ == "__main__":
    main()
