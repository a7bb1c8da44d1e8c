"""c5 timing: lib/spm_train --model_type=unigram --vocab_size=32000 on N
synthetic lines (tools/synth.py, the c2 distribution), written to a temp
file first.  Prints the trainer's --timings JSON line plus the corpus size.

  python tools/train_bench.py --lines 1000000 [--vocab 32000] [--args "..."]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402

TRAIN = os.path.join(ROOT, "sentencepiece-comments_amd", "lib", "spm_train")


def _chunk_bytes(args):
    """Lines [start, start + m) of the corpus (seed + start), newline-terminated."""
    import numpy as np
    start, m, seed = args
    buf, off = synth.raw(m, seed=seed + start)
    return np.insert(buf, off[1:].astype(np.int64), 10).tobytes()


def write_corpus(path, n, seed, chunk=5_000_000, workers=1):
    """The same bytes for any `workers`: chunk k is drawn with seed + k*chunk.
    workers > 1 draws chunks in a process pool (call this from a process that
    has not initialised the GPU)."""
    jobs = [(start, min(chunk, n - start), seed) for start in range(0, n, chunk)]
    with open(path, "wb") as f:
        if workers > 1 and len(jobs) > 1:
            import multiprocessing as mp
            with mp.get_context("spawn").Pool(min(workers, len(jobs))) as pool:
                for k, b in enumerate(pool.imap(_chunk_bytes, jobs)):
                    f.write(b)
                    print("corpus: %d / %d lines" % (jobs[k][0] + jobs[k][1], n), file=sys.stderr, flush=True)
        else:
            for j in jobs:
                f.write(_chunk_bytes(j))
                if n > chunk:
                    print("corpus: %d / %d lines" % (j[0] + j[1], n), file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=1_000_000)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--args", default="--normalization_rule_name=identity --num_threads=16")
    ap.add_argument("--keep", default="")
    ap.add_argument("--log", default="", help="stream the trainer's stderr to this file")
    ap.add_argument("--workers", type=int, default=1, help="processes drawing the synthetic corpus")
    ap.add_argument("--model-type", default="unigram")
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="spm_c5_")
    corpus = os.path.join(d, "corpus.txt")
    t0 = time.time()
    write_corpus(corpus, a.lines, a.seed, workers=a.workers)
    gen_s = time.time() - t0
    prefix = a.keep or os.path.join(d, "m")
    cmd = [TRAIN, "--input=" + corpus, "--model_prefix=" + prefix, "--model_type=" + a.model_type,
           "--vocab_size=%d" % a.vocab, "--timings"] + a.args.split()
    t0 = time.time()
    err = open(a.log, "ab") if a.log else subprocess.PIPE
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=err)
    wall = time.time() - t0
    if p.returncode != 0:
        if not a.log:
            sys.stderr.write(p.stderr.decode(errors="replace")[-4000:])
        sys.exit(p.returncode)
    tm = json.loads(p.stdout.decode().strip().splitlines()[-1])
    tm.update({"lines": a.lines, "corpus_bytes": os.path.getsize(corpus), "gen_s": gen_s,
               "wall_s": wall, "vocab": a.vocab})
    if not a.log:
        # The load breakdown and the whitespace split's path (device, or the
        # host fallback and why).
        log = p.stderr.decode(errors="replace").splitlines()
        tm["split_log"] = [l for l in log if "split" in l][-3:]
        tm["load_log"] = [l for l in log if l.startswith("LoadSentences")][-1:]
    print(json.dumps(tm))
    os.remove(corpus)


if __name__ == "__main__":
    main()
