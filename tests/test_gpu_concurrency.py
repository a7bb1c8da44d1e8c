"""One model handle shared by many host threads (the reference's contract:
unigram::Model::Encode / bpe::Model::Encode are const and keep their lattice /
agenda on the stack, unigram_model.cc:705-720, bpe_model.cc:37-199, so one
SentencePieceProcessor serves every thread).

8 host threads × 2 streams each encode different batches through ONE
spm_hip_model; half of them also call the host-buffer entry point.  Every
result must be bit-exact against the oracle.
"""
import os
import threading

import numpy as np
import pytest

import oracle_lib as O
import spm_amd as S
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

THREADS, STREAMS, ROUNDS = 8, 2, 3


@pytest.mark.parametrize("model_name", ["synth32k_unigram.model", "synth32k_bpe.model"])
def test_one_handle_many_threads_and_streams(model_name):
    import torch
    dev = torch.device("cuda", 0)
    mb = open(os.path.join(ROOT, "data", model_name), "rb").read()
    om = O.OracleModel(mb)
    batches, want = [], []
    for k in range(THREADS * STREAMS):
        buf, off = synth.normalized(3000 + 997 * k, seed=500 + k)
        batches.append((buf, off))
        ids, lens, to = om.encode_normalized_csr(buf, off, threads=8, with_lens=True)
        want.append((ids, lens, to))
    dm = S.DeviceModel(mb)
    errors = []
    start = threading.Barrier(THREADS)

    def worker(t):
        try:
            torch.cuda.set_device(dev)
            streams = [torch.cuda.Stream(dev) for _ in range(STREAMS)]
            start.wait()
            for r in range(ROUNDS):
                pending = []
                for j, s in enumerate(streams):
                    k = t * STREAMS + j
                    buf, off = batches[k]
                    n = len(off) - 1
                    with torch.cuda.stream(s):
                        d_b = torch.from_numpy(buf).to(dev, non_blocking=False)
                        d_o = torch.from_numpy(off.view(np.int64)).to(dev)
                        d_ids = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=dev)
                        d_len = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=dev)
                        d_tok = torch.empty(n + 1, dtype=torch.int64, device=dev)
                    dm.encode_device(d_b.data_ptr(), d_o.data_ptr(), n, d_ids.data_ptr(), d_tok.data_ptr(),
                                     d_len=d_len.data_ptr(), stream=s.cuda_stream)
                    pending.append((k, s, d_b, d_o, d_ids, d_len, d_tok))
                if t % 2 == 1:  # host-buffer API interleaved with the device calls
                    k = (t * STREAMS + r) % len(batches)
                    buf, off = batches[k]
                    ids, lens, to = dm.encode_csr_host(buf, off, with_lens=True)
                    wi, wl, wt = want[k]
                    if not (np.array_equal(to, wt) and np.array_equal(ids, wi) and np.array_equal(lens, wl)):
                        errors.append("host api thread %d round %d batch %d" % (t, r, k))
                for k, s, d_b, d_o, d_ids, d_len, d_tok in pending:
                    s.synchronize()
                    to = d_tok.cpu().numpy().view(np.uint64)
                    ntok = int(to[-1])
                    ids = d_ids[:ntok].cpu().numpy()
                    lens = d_len[:ntok].cpu().numpy().view(np.uint32)
                    wi, wl, wt = want[k]
                    if not (np.array_equal(to, wt) and np.array_equal(ids, wi) and np.array_equal(lens, wl)):
                        errors.append("device api thread %d round %d batch %d" % (t, r, k))
        except Exception as e:  # noqa: BLE001 — reported below
            errors.append("thread %d: %r" % (t, e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=100)
    assert not any(x.is_alive() for x in th), "worker hung"
    assert not errors, errors[:5]
