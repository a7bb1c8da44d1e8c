"""Train the 32k synthetic unigram / BPE models used by the c2/c3 benchmarks.

Trained with the installed reference-family pip `sentencepiece` (v0.2.2) on the
first 1M lines of tools/synth.py (seed 1234), vocab 32000, num_threads 8,
default (nmt_nfkc) normalization.  The resulting .model files are committed
under data/; encode parity is always checked against the CPU oracle on the
same model, so the trainer used to make them does not matter for parity.
"""
import os
import sys
import tempfile

import sentencepiece as spm

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import synth  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "data")


def main():
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "synth1m.txt")
        with open(path, "wb") as f:
            for ln in synth.lines(1000000):
                f.write(ln + b"\n")
        for mt in ("unigram", "bpe"):
            prefix = os.path.join(d, "synth32k_" + mt)
            spm.SentencePieceTrainer.train(
                input=path, model_prefix=prefix, vocab_size=32000, model_type=mt,
                num_threads=8, input_sentence_size=1000000, shuffle_input_sentence=False,
                minloglevel=2)
            os.replace(prefix + ".model", os.path.join(OUT, "synth32k_%s.model" % mt))


if __name__ == "__main__":
    main()
