"""Full-size check of the seed miner's first-symbol split (seed_kernels.hip,
corpora of >= 2^28 chars): lib/spm_train on the c5 corpus (100 M synthetic
lines, tools/train_bench.py) twice, SPM_HIP_SEED_PARTS=1 (one LSD order over
all suffixes) and the default (4 parts); the dumped seed lists (piece, float
bits) and the .model piece tables and .vocab files must be identical.  Prints one JSON line.

  python tools/seed_split_check.py [--lines 100000000] [--workers 16]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import model_reader  # noqa: E402
import train_bench as tb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=100_000_000)
    ap.add_argument("--workers", type=int, default=16)
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="spm_split_")
    corpus = os.path.join(d, "corpus.txt")
    tb.write_corpus(corpus, a.lines, 1234, workers=a.workers)
    out = {"lines": a.lines, "corpus_bytes": os.path.getsize(corpus)}
    digests = {}
    for parts in ("1", "default"):
        env = dict(os.environ)
        if parts == "1":
            env["SPM_HIP_SEED_PARTS"] = "1"
        else:
            env.pop("SPM_HIP_SEED_PARTS", None)
        prefix = os.path.join(d, "m" + parts)
        seeds = prefix + ".seeds"
        cmd = [tb.TRAIN, "--input=" + corpus, "--model_prefix=" + prefix, "--model_type=unigram",
               "--vocab_size=32000", "--timings", "--dump_seeds=" + seeds,
               "--normalization_rule_name=identity", "--num_threads=16"]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)
        if p.returncode != 0:
            sys.stderr.write(p.stderr.decode(errors="replace")[-3000:])
            sys.exit(1)
        tm = json.loads(p.stdout.decode().strip().splitlines()[-1])
        digests[parts] = {
            "seeds_sha256": hashlib.sha256(open(seeds, "rb").read()).hexdigest(),
            # (the .model's trainer spec holds the prefix: compare its piece table and the .vocab)
            "pieces_sha256": hashlib.sha256(repr(model_reader.read_pieces(
                open(prefix + ".model", "rb").read())).encode()).hexdigest(),
            "vocab_sha256": hashlib.sha256(open(prefix + ".vocab", "rb").read()).hexdigest(),
            "seed_s": tm.get("seed_s"), "total_s": tm.get("total_s"),
            "seed_peak_bytes": (tm.get("stage_peak_bytes") or [None, None])[1],
            "seed_stages_ms": tm.get("seed_stages_ms"),
        }
        print("parts=%s %s" % (parts, json.dumps(digests[parts])), file=sys.stderr, flush=True)
    out["runs"] = digests
    out["seeds_identical"] = digests["1"]["seeds_sha256"] == digests["default"]["seeds_sha256"]
    out["model_identical"] = all(digests["1"][k] == digests["default"][k] for k in ("pieces_sha256", "vocab_sha256"))
    print(json.dumps(out))
    sys.exit(0 if out["seeds_identical"] and out["model_identical"] else 2)


if __name__ == "__main__":
    main()
