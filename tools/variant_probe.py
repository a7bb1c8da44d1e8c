"""Encode one golden corpus with one unigram kernel variant and compare with
the oracle (debug tool; run one variant per process under a timeout)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sentencepiece-comments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch  # noqa: F401  (binds the library to torch's HIP runtime)
import spm_amd as S
import oracle_lib as O

variant, model, text = sys.argv[1], sys.argv[2], sys.argv[3]
limit = int(sys.argv[4]) if len(sys.argv) > 4 else 0
os.environ["SPM_HIP_UNIGRAM_VARIANT"] = variant
mb = open(os.path.join(ROOT, model), "rb").read()
lines = O.read_lines_binary(os.path.join(ROOT, text))
om = O.OracleModel(mb)
norm = om.normalize(lines)
if limit:
    norm = [s for s in norm if len(s) <= limit]
buf, off = S.to_csr(norm)
print("variant", variant, "sentences", len(norm), "max bytes", max(len(s) for s in norm), flush=True)
dm = S.DeviceModel(mb)
print("fast_variant", dm.info().fast_variant, flush=True)
t = time.time()
ids, lens, to = dm.encode_csr_host(buf, off, with_lens=True)
print("encoded in %.3f s, general %d" % (time.time() - t, dm.stats().general_path), flush=True)
oids, olens, oto = om.encode_normalized_csr(buf, off, threads=8, with_lens=True)
print("match", np.array_equal(to, oto) and np.array_equal(ids, oids) and np.array_equal(lens, olens), flush=True)
