"""The pure stream entry points (spm_hip_*_async): same results as the
blocking calls, no host synchronization, errors through the device status
word (first error wins, later calls of the chain do nothing)."""
import os

import numpy as np
import pytest

import oracle_lib as O
import spm_amd as S
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(ROOT, "data")

pytestmark = pytest.mark.gpu


def _read(p):
    return open(p, "rb").read()


def _dev():
    import torch
    return torch.device("cuda", torch.cuda.current_device())


def _encode_async(dm, sents, capacity=None, status_init=0, with_lens=False):
    import torch
    dev = _dev()
    buf, off = S.to_csr(sents)
    n = len(sents)
    cap = int(off[-1]) if capacity is None else capacity
    d_b = torch.from_numpy(buf).to(dev)
    d_o = torch.from_numpy(off.view(np.int64)).to(dev)
    d_ids = torch.full((max(int(off[-1]), cap, 1),), -7, dtype=torch.int32, device=dev)
    d_len = torch.zeros(max(int(off[-1]), cap, 1), dtype=torch.int32, device=dev) if with_lens else None
    d_tok = torch.full((n + 1,), -7, dtype=torch.int64, device=dev)
    d_st = torch.full((1,), status_init, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    dm.encode_device_async(d_b.data_ptr(), d_o.data_ptr(), n, cap, d_ids.data_ptr(), d_tok.data_ptr(),
                           d_st.data_ptr(), d_len=d_len.data_ptr() if with_lens else None, stream=s)
    torch.cuda.synchronize(dev)
    tok = d_tok.cpu().numpy().view(np.uint64)
    k = int(tok[-1]) if int(d_st.item()) == 0 else 0
    lens = d_len[:k].cpu().numpy().view(np.uint32) if with_lens else None
    return d_ids[:k].cpu().numpy(), tok, int(d_st.item()), lens, d_ids.cpu().numpy()


@pytest.mark.parametrize("kind", ["unigram", "bpe"])
def test_async_equals_blocking(kind):
    mb = _read(os.path.join(DATA, "synth32k_%s.model" % kind))
    buf, off = synth.normalized(20000, seed=31)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)] + ["▁".encode() + b"xyz" * 40]
    dm = S.DeviceModel(mb)
    ids, tok, st, lens, _ = _encode_async(dm, sents, with_lens=True)
    assert st == 0
    bbuf, boff = S.to_csr(sents)
    rids, rlens, rtok = dm.encode_csr_host(bbuf, boff, with_lens=True)
    assert np.array_equal(tok, rtok) and np.array_equal(ids, rids) and np.array_equal(lens, rlens)


def test_async_flagged_sentences_fixup():
    """Sentences the fast kernel flags (0xFF bytes, broken UTF-8, the debug
    back-pointer knob) go through the device-count general pass and the
    fix-up chain in the asynchronous call too: bit-exact vs the oracle."""
    mb = _read(os.path.join(DATA, "synth32k_unigram.model"))
    buf, off = synth.normalized(5000, seed=32)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    for k in range(0, 5000, 97):
        sents[k] = sents[k] + b"\xff" + sents[k][:5]
    sents[10] = b"\xe3\x81" + sents[10]
    dm = S.DeviceModel(mb)
    dm.set_debug_corrupt_bp(2000)
    ids, tok, st, lens, _ = _encode_async(dm, sents, with_lens=True)
    assert st == 0
    bbuf, boff = S.to_csr(sents)
    oids, olens, otok = O.OracleModel(mb).encode_normalized_csr(bbuf, boff, threads=8, with_lens=True)
    assert np.array_equal(tok, otok) and np.array_equal(ids, oids) and np.array_equal(lens, olens)


@pytest.mark.parametrize("kind", ["unigram", "bpe"])
def test_async_capacity_exceeded(kind):
    """offsets[n] > capacity: RESOURCE_EXHAUSTED in the status word, nothing
    written past the caller's buffers, and the stream keeps working."""
    mb = _read(os.path.join(DATA, "synth32k_%s.model" % kind))
    buf, off = synth.normalized(2000, seed=33)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    dm = S.DeviceModel(mb)
    _, _, st, _, raw = _encode_async(dm, sents, capacity=int(off[-1]) // 2)
    assert st == 8
    ids, tok, st2, _, _ = _encode_async(dm, sents)
    assert st2 == 0
    rids, rtok = dm.encode_csr_host(*S.to_csr(sents))
    assert np.array_equal(ids, rids) and np.array_equal(tok, rtok)


def test_async_status_set_means_noop():
    """A non-zero status word (an earlier failure of the chain) turns every
    later asynchronous call into a no-op: outputs stay untouched."""
    mb = _read(os.path.join(DATA, "synth32k_unigram.model"))
    buf, off = synth.normalized(1000, seed=34)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    _, tok, st, _, raw = _encode_async(S.DeviceModel(mb), sents, status_init=13)
    assert st == 13
    assert (raw == -7).all() and (tok.view(np.int64) == -7).all()


def test_async_general_overflow_and_blocking_rerun():
    """A flagged sentence longer than the device general pass's scratch
    (> 256 KiB): the asynchronous call reports RESOURCE_EXHAUSTED; the
    blocking call re-runs the batch with host-sized scratch, bit-exact."""
    mb = _read(os.path.join(DATA, "synth32k_unigram.model"))
    rng = np.random.default_rng(35)
    words = [b"the", b"a", b"piece", b"of", b"text", b"and", b"more"]
    big = b"".join("▁".encode() + words[int(x)] for x in rng.integers(0, len(words), 60000))
    big = big[:150000] + b"\xff" + big[150000:300000]
    sents = [b"\xe2\x96\x81hello", big, "▁short".encode()]
    dm = S.DeviceModel(mb)
    _, _, st, _, _ = _encode_async(dm, sents)
    assert st == 8
    bbuf, boff = S.to_csr(sents)
    ids, lens, tok = dm.encode_csr_host(bbuf, boff, with_lens=True)
    oids, olens, otok = O.OracleModel(mb).encode_normalized_csr(bbuf, boff, threads=1, with_lens=True)
    assert np.array_equal(tok, otok) and np.array_equal(ids, oids) and np.array_equal(lens, olens)
    assert dm.stats().general_path == len(sents)  # the host-sized re-run


@pytest.mark.parametrize("model_name,text", [
    ("test_model.model", "botchan.txt"),
    ("botchan_bpe1k.model", "botchan.txt"),
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt"),
])
@pytest.mark.parametrize("opts", ["", "bos:eos", "reverse:bos"])
def test_async_raw_chain_equals_blocking(model_name, text, opts):
    """normalize_async -> encode_async -> finalize_ids_async on one stream
    with one status word == the blocking device pipeline == the oracle."""
    mb = _read(os.path.join(GOLD, model_name))
    lines = O.read_lines_binary(os.path.join(GOLD, text))[:1200] + [b"", b" ", "▁".encode()]
    dm = S.DeviceModel(mb)
    got, code = dm.encode_lines_device_async(lines, opts)
    assert code == 0
    om = O.OracleModel(mb)
    om.set_extra_options(opts)
    assert got == om.encode_lines(lines)


def test_drain_kernel_times_and_stream_pool():
    """Fast-kernel event times of asynchronous calls are drained per stream;
    more streams than the pool bound (16) recycle workspaces and stay exact."""
    import torch
    dev = _dev()
    mb = _read(os.path.join(DATA, "synth32k_unigram.model"))
    buf, off = synth.normalized(4000, seed=36)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    dm = S.DeviceModel(mb)
    dm.set_timing(True)
    want, wtok = dm.encode_csr_host(*S.to_csr(sents))
    s0 = torch.cuda.current_stream(dev).cuda_stream
    dm.drain_kernel_times(s0)
    for _ in range(3):
        ids, tok, st, _, _ = _encode_async(dm, sents)
        assert st == 0 and np.array_equal(ids, want)
    t = dm.drain_kernel_times(s0)
    assert len(t) == 3 and all(x > 0 for x in t)
    streams = [torch.cuda.Stream(device=dev) for _ in range(20)]
    for sk in streams:
        with torch.cuda.stream(sk):
            ids, tok, st, _, _ = _encode_async(dm, sents)
            assert st == 0 and np.array_equal(ids, want) and np.array_equal(tok, wtok)
    dm.release_stream(streams[-1].cuda_stream)


def test_async_force_general_status_set_means_noop():
    """Host-sized models (here force_general) run the general kernel with
    host-sized scratch; a status word an earlier call of the chain already
    set still turns the call into a no-op (it used to launch and
    overwrite the word)."""
    mb = _read(os.path.join(DATA, "synth32k_unigram.model"))
    buf, off = synth.normalized(500, seed=37)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    dm = S.DeviceModel(mb)
    dm.set_force_general(True)
    _, tok, st, _, raw = _encode_async(dm, sents, status_init=13)
    assert st == 13
    assert (raw == -7).all() and (tok.view(np.int64) == -7).all()
    ids, tok, st, _, _ = _encode_async(dm, sents)
    assert st == 0
    rids, rtok = O.OracleModel(mb).encode_normalized_csr(*S.to_csr(sents), threads=4)
    assert np.array_equal(ids, rids) and np.array_equal(tok, rtok)


def test_async_force_general_after_normalize_overflow():
    """normalize_async into a too-small buffer (RESOURCE_EXHAUSTED, offsets
    past the buffer) -> encode_async of a host-sized model: nothing is read
    or written, the first error stays in the status word."""
    import torch
    dev = _dev()
    mb = _read(os.path.join(GOLD, "test_model.model"))
    lines = O.read_lines_binary(os.path.join(GOLD, "botchan.txt"))[:300]
    dm = S.DeviceModel(mb)
    dm.set_force_general(True)
    buf, off = S.to_csr(lines)
    n = len(lines)
    cap = int(off[-1]) // 4
    d_in = torch.from_numpy(buf).to(dev)
    d_in_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_norm = torch.zeros(cap, dtype=torch.uint8, device=dev)
    d_noff = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_ids = torch.full((cap,), -7, dtype=torch.int32, device=dev)
    d_tok = torch.full((n + 1,), -7, dtype=torch.int64, device=dev)
    d_st = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    dm.normalize_device_async(d_in.data_ptr(), d_in_off.data_ptr(), n, d_norm.data_ptr(), cap, d_noff.data_ptr(),
                              d_st.data_ptr(), stream=s)
    dm.encode_device_async(d_norm.data_ptr(), d_noff.data_ptr(), n, cap, d_ids.data_ptr(), d_tok.data_ptr(),
                           d_st.data_ptr(), stream=s)
    torch.cuda.synchronize(dev)
    assert int(d_st.item()) == 8
    assert (d_ids.cpu().numpy() == -7).all() and (d_tok.cpu().numpy() == -7).all()
