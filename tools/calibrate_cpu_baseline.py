"""Calibrates the bench's CPU baseline (the oracle port, oracle/spm_oracle.cc)
against a reference-family build: pip sentencepiece 0.2.2 (importable in the
build container, not on the GPU box), on the SAME inputs, at 1 and N threads.

Two comparisons on the c2 generator (tools/synth.py):
  model-only : normalized sentences -> ids.  Oracle: Model::Encode
               restatement (encode_normalized_csr, strided threads).  pip:
               SentencePieceProcessor.Encode on the same normalized bytes with
               the c2 model's pieces under an identity NormalizerSpec (no
               charsmap, no dummy prefix, no whitespace rewriting), so its
               normalizer pass is a copy.
  full       : raw lines -> ids (Normalizer + Encode + epilogue), 1 thread.
Prints one JSON line; DESIGN.md §5 and bench.py's cpu_baseline note quote it.

  python tools/calibrate_cpu_baseline.py [--sentences 500000] [--threads 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sentences", type=int, default=500_000)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    import numpy as np
    import sentencepiece as spm
    import model_builder
    import model_reader
    import oracle_lib
    import synth
    mb = open(os.path.join(ROOT, "data", "synth32k_unigram.model"), "rb").read()
    pieces = model_reader.read_pieces(mb)
    ident = model_builder.model(pieces, model_builder.UNIGRAM, charsmap=b"", add_dummy_prefix=False,
                                remove_extra_whitespaces=False, escape_whitespaces=True)
    n = args.sentences
    buf, off = synth.normalized(n, seed=4321)
    b = buf.tobytes()
    norm = [b[int(off[i]):int(off[i + 1])].decode() for i in range(n)]
    om = oracle_lib.OracleModel(mb)
    res = {"sentences": n, "pip_sentencepiece": spm.__version__, "cpus": os.cpu_count()}

    def timeit(f):
        t0 = time.perf_counter()
        out = f()
        return time.perf_counter() - t0, out

    sp_id = spm.SentencePieceProcessor(model_proto=ident)
    for th in (1, args.threads):
        dt_o, (oids, oto) = timeit(lambda: om.encode_normalized_csr(buf, off, threads=th))
        dt_p, pids = timeit(lambda: sp_id.encode(norm, num_threads=th))
        res["model_only_t%d" % th] = {"oracle_sent_per_s": n / dt_o, "pip_sent_per_s": n / dt_p,
                                      "oracle_over_pip": dt_p / dt_o}
    # Parity of the two on this corpus (no UNK merges occur in it).  0.2.2's
    # unigram Encode resolves exact float ties of the Viterbi score
    # differently from v0.1.82 (first lnode wins, unigram_model.cc:240-245):
    # every sentence whose ids differ is checked to be such a tie (the two
    # segmentations' scores, summed in float left to right, are bit-equal).
    flat = np.fromiter((x for r in pids for x in r), dtype=np.int32)
    res["model_only_ids_equal"] = bool(np.array_equal(flat, oids))
    score = np.array([s for _, s, _ in pieces], dtype=np.float32)

    def fsum(ids):
        acc = np.float32(0)
        for x in ids:
            acc = np.float32(acc + score[x])
        return acc

    diff = ties = 0
    for i in range(n):
        o = oids[oto[i]:oto[i + 1]].tolist()
        if o != list(pids[i]):
            diff += 1
            ties += int(fsum(o) == fsum(pids[i]))
    res["model_only_diff_sentences"] = diff
    res["model_only_diff_exact_float_ties"] = ties
    # Full pipeline on raw lines (the oracle's encode_lines is single-threaded).
    m = n // 5
    rbuf, roff = synth.raw(m, seed=4321)
    rb = rbuf.tobytes()
    raw = [rb[int(roff[i]):int(roff[i + 1])] for i in range(m)]
    sp_full = spm.SentencePieceProcessor(model_proto=mb)
    dt_o, olines = timeit(lambda: om.encode_lines(raw))
    dt_p, plines = timeit(lambda: sp_full.encode([r.decode() for r in raw], num_threads=1))
    res["full_t1"] = {"sentences": m, "oracle_sent_per_s": m / dt_o, "pip_sent_per_s": m / dt_p,
                      "oracle_over_pip": dt_p / dt_o, "ids_equal": olines == plines,
                      "diff_sentences": sum(int(list(a) != list(b)) for a, b in zip(olines, plines))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
