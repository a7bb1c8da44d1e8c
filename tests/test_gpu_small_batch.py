"""Small host batches (spm_hip_encode_batch_host with n <= 256: the single
tile path, one upload and one synchronization; a flagged sentence takes a
second round trip through the general kernel and the fix-up chain) stay
bit-exact against the oracle, including empty sentences, an all-empty batch,
flagged sentences and the 256/257 boundary."""
import os

import numpy as np
import pytest

import oracle_lib as O
import spm_amd as S
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _sents(n, seed):
    buf, off = synth.normalized(n, seed=seed)
    b = buf.tobytes()
    return [b[int(off[i]):int(off[i + 1])] for i in range(n)]


@pytest.mark.parametrize("model", ["synth32k_unigram.model", "synth32k_bpe.model"])
def test_small_batches_exact(model):
    mb = open(os.path.join(ROOT, "data", model), "rb").read()
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    pool = _sents(3000, 41)
    pool[5] = pool[5] + b"\xff" + pool[5][:4]          # flagged by the byte kernel
    pool[300] = b"\xe3\x81" + pool[300]                # broken UTF-8
    pool[7] = b""
    start = 0
    for n in (1, 2, 3, 17, 255, 256, 257, 1, 64):
        batch = pool[start:start + n]
        start += n
        buf, off = S.to_csr(batch)
        ids, lens, tok = dm.encode_csr_host(buf, off, with_lens=True)
        rids, rlens, rtok = om.encode_normalized_csr(buf, off, with_lens=True)
        assert np.array_equal(tok, rtok) and np.array_equal(ids, rids) and np.array_equal(lens, rlens), n
    # single flagged sentence alone, and an all-empty batch
    for batch in ([pool[5]], [b"", b""], [b"\xff"]):
        buf, off = S.to_csr(batch)
        ids, lens, tok = dm.encode_csr_host(buf, off, with_lens=True)
        rids, rlens, rtok = om.encode_normalized_csr(buf, off, with_lens=True)
        assert np.array_equal(tok, rtok) and np.array_equal(ids, rids) and np.array_equal(lens, rlens), batch
    dm.close()
