"""Writes data/normalization/<rule>.bin: precompiled charsmap blobs for
spm_train --normalization_rule_name (reference Builder::GetPrecompiledCharsMap,
builder.cc:280-299; the reference's normalization_rule.h is missing from its
tree, .MISSING_LARGE_BLOBS).

  nfkc     : the charsmap embedded in the reference's own test model
             python/test/test_model.model (tests/golden/test_model.model) —
             reference-era NFKC.
  nmt_nfkc : the charsmap embedded in data/synth32k_unigram.model, which the
             installed pip sentencepiece 0.2.2 wrote (a SUBSTITUTE, not the
             reference-era blob; parity tests use identity or nfkc).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import model_reader  # noqa: E402

SOURCES = {
    "nfkc": os.path.join(ROOT, "tests", "golden", "test_model.model"),
    "nmt_nfkc": os.path.join(ROOT, "data", "synth32k_unigram.model"),
}


def main():
    out = os.path.join(ROOT, "data", "normalization")
    os.makedirs(out, exist_ok=True)
    for name, src in SOURCES.items():
        blob = model_reader.charsmap(open(src, "rb").read())
        open(os.path.join(out, name + ".bin"), "wb").write(blob)
        print(name, len(blob))


if __name__ == "__main__":
    main()
