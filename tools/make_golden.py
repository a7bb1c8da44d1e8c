"""Generate golden id fixtures for the encode path (test infrastructure).

Inputs are the reference's own fixtures, copied verbatim into tests/golden/:
  botchan.txt, wagahaiwa_nekodearu.txt  (data/ in the reference)
  test_model.model, test_ja_model.model (python/test/ in the reference)

The reference C++ tree cannot be built here under the round rules (it needs
the cmake-generated config.h), so the ids are produced with the installed
reference-family pip `sentencepiece` (v0.2.2) exactly as `spm_encode
--output_format=id` would: one line at a time, read in binary mode keeping
'\r' (filesystem.cc:42-44 uses std::getline).  tests/test_oracle_golden.py then
checks the CPU oracle against these files line by line.

Usage: python tools/make_golden.py
"""
import hashlib
import os
import sys

import sentencepiece as spm

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "..", "tests", "golden")


def encode_file(model, text, out, pieces=False):
    sp = spm.SentencePieceProcessor()
    sp.LoadFromSerializedProto(open(os.path.join(GOLD, model), "rb").read())
    data = open(os.path.join(GOLD, text), "rb").read()
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    with open(os.path.join(GOLD, out), "w") as f:
        for ln in lines:
            # EncodeAsIds takes str; decode with surrogateescape is not needed
            # for these UTF-8 corpora.
            if pieces:
                f.write(" ".join(sp.EncodeAsPieces(ln.decode("utf-8"))) + "\n")
            else:
                ids = sp.EncodeAsIds(ln.decode("utf-8"))
                f.write(" ".join(map(str, ids)) + "\n")
    h = hashlib.sha256(open(os.path.join(GOLD, out), "rb").read()).hexdigest()
    print(out, len(lines), "lines sha256", h, "spm", spm.__version__)


if __name__ == "__main__":
    encode_file("test_model.model", "botchan.txt", "botchan_test_model.ids")
    encode_file("test_ja_model.model", "wagahaiwa_nekodearu.txt", "wagahaiwa_test_ja_model.ids")
    # 1k BPE model trained on botchan with the same pip sentencepiece (committed).
    encode_file("botchan_bpe1k.model", "botchan.txt", "botchan_bpe1k.ids")
    # --output_format=piece (survey: sha256 b8a30920...5209 with the reference build).
    encode_file("test_model.model", "botchan.txt", "botchan_test_model.pieces", pieces=True)
