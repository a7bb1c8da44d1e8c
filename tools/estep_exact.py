"""Diagnostic: exact-mismatch census of the PARITY E-step vs the oracle.

Prints, per (corpus, T), the number of expected[] entries that differ from the
oracle's, the obj / ntok equality, and for the first few mismatching pieces the
float values and their ulp distance.  GPU box only (loads libspm_hip.so).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "sentencepiece-comments_amd", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))
import model_reader  # noqa: E402
import oracle_lib as O  # noqa: E402
import spm_amd as S  # noqa: E402
import synth  # noqa: E402


def pieces_of(path):
    pcs = [(p, s) for p, s, t in model_reader.read_pieces(open(path, "rb").read()) if t == 1]
    return [p for p, _ in pcs], np.array([s for _, s in pcs], dtype=np.float32)


def census(tag, sents, freqs, pieces, scores, T):
    e_ref, o_ref, n_ref = O.estep(sents, freqs, pieces, scores, T)
    dp = S.DevicePieces(pieces, scores)
    e, o, n = dp.estep(sents, freqs, mode=S.SPM_ESTEP_PARITY, threads=T)
    bad = np.nonzero(e.view(np.uint32) != e_ref.view(np.uint32))[0]
    print("%s T=%d n=%d mismatches=%d/%d obj_eq=%s (%r vs %r) ntok_eq=%s" %
          (tag, T, len(sents), len(bad), len(e), o == o_ref, float(o), float(o_ref), n == n_ref), flush=True)
    for i in bad[:8]:
        ulp = int(e.view(np.int32)[i]) - int(e_ref.view(np.int32)[i])
        print("   piece %d %r: dev %r ref %r ulp %d" % (i, pieces[i], float(e[i]), float(e_ref[i]), ulp))


def main():
    pieces, scores = pieces_of(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    buf, off = synth.normalized(60000, seed=5)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(60000)]
    freqs = np.random.default_rng(5).integers(1, 4, size=60000)
    for T in (1, 8, 16):
        census("synth60k", sents, freqs, pieces, scores, T)
    gp, gs = pieces_of(os.path.join(ROOT, "tests", "golden", "test_model.model"))
    mb = open(os.path.join(ROOT, "tests", "golden", "test_model.model"), "rb").read()
    lines = O.read_lines_binary(os.path.join(ROOT, "tests", "golden", "botchan.txt"))
    bs = [s for s in O.OracleModel(mb).normalize(lines) if s]
    bs += [b"\xff\xfeabc", "é".encode() + b"\x80z", b"a" * 300]
    bf = np.arange(len(bs)) % 5 + 1
    for T in (1, 16):
        census("botchan", bs, bf, gp, gs, T)


if __name__ == "__main__":
    main()
