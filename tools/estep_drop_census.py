"""Writes the c4 inputs for tools/estep_drop_census.cc (diagnostic only):
N synthetic normalized sentences (tools/synth.py, seed 99 as bench.py's
E-step leg) and the NORMAL pieces of data/synth32k_unigram.model.
Usage: python tools/estep_drop_census.py DIR [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import model_reader  # noqa: E402
import synth  # noqa: E402

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
os.makedirs(d, exist_ok=True)
buf, off = synth.normalized(n, seed=99)
buf.tofile(os.path.join(d, "sent.bin"))
off.astype(np.uint64).tofile(os.path.join(d, "sent_off.bin"))
pcs = [(p, s) for p, s, t in model_reader.read_pieces(open(os.path.join(ROOT, "data", "synth32k_unigram.model"), "rb").read()) if t == 1]
pb = b"".join(p if isinstance(p, bytes) else p.encode() for p, _ in pcs)
po = np.zeros(len(pcs) + 1, dtype=np.uint64)
po[1:] = np.cumsum([len(p if isinstance(p, bytes) else p.encode()) for p, _ in pcs])
open(os.path.join(d, "pieces.bin"), "wb").write(pb)
po.tofile(os.path.join(d, "piece_off.bin"))
np.array([s for _, s in pcs], dtype=np.float32).tofile(os.path.join(d, "scores.bin"))
print("wrote", n, "sentences,", len(pcs), "pieces")
