"""GPU parity of the unigram trainer E-step (RunEStep) vs the CPU oracle.

PARITY mode is asserted bit-exact (expected[], obj, ntok) against the oracle's
T-bucket emulation of RunEStep (unigram_model_trainer.cc:237-287), which
SURVEY §8a E1 measured bit-identical to the real RunEStep at T = 1, 8, 16.
The only theoretical deviation is a device-vs-glibc exp/log ulp: every such
double result is rounded to float (LogSumExp's return, `float += double`), so
a 1-ulp double difference flips a float only when it lies within one double
ulp of a float rounding midpoint (about 2^-29 per operation); none has been
observed on any corpus here (tools/estep_exact.py census).
"""
import os

import numpy as np
import pytest

import known_answers as KA
import oracle_lib as O
import spm_amd as S
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _pieces_from_model(path, normal_only=True):
    """TrainerModel piece list = the NORMAL pieces of a model, in order."""
    import model_reader
    pcs = model_reader.read_pieces(open(path, "rb").read())
    keep = [(p, s) for (p, s, t) in pcs if (t == 1 or not normal_only)]
    return [p for p, _ in keep], np.array([s for _, s in keep], dtype=np.float32)


def _corpus(n, seed):
    buf, off = synth.normalized(n, seed=seed)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(n)]
    rng = np.random.default_rng(seed)
    freqs = rng.integers(1, 4, size=n)
    return sents, freqs


# spm_hip_pieces_set_forward: 1 = the encode byte kernel's E-step mode (the
# default for calls of >= 2^20 sentences), 2 = estep_forward_kernel.
FORWARDS = [1, 2]


def _assert_exact(sents, freqs, pieces, scores, threads, forward=0):
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, threads)
    dp = S.DevicePieces(pieces, scores)
    dp.set_forward(forward)
    e, obj, nt = dp.estep(sents, freqs, mode=S.SPM_ESTEP_PARITY, threads=threads)
    bad = np.nonzero(e.view(np.uint32) != e_ref.view(np.uint32))[0]
    assert len(bad) == 0, ("inexact pieces", len(bad), [(int(i), float(e[i]), float(e_ref[i]))
                                                        for i in bad[:5]])
    assert np.float32(obj).view(np.uint32) == np.float32(obj_ref).view(np.uint32), (obj, obj_ref)
    assert nt == nt_ref
    return e, obj, nt


def _check_close(got, ref):
    nz = ref != 0
    rel = np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])
    assert np.all(got[~nz] == 0)
    return float(rel.max()) if rel.size else 0.0


@pytest.mark.parametrize("forward", FORWARDS)
@pytest.mark.parametrize("threads", [1, 8, 16])
def test_estep_parity_mode(threads, forward):
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    sents, freqs = _corpus(60000, 5)
    _assert_exact(sents, freqs, pieces, scores, threads, forward)


@pytest.mark.parametrize("forward", FORWARDS)
def test_estep_fast_mode(forward):
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    sents, freqs = _corpus(60000, 6)
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, 1)
    dp = S.DevicePieces(pieces, scores)
    dp.set_forward(forward)
    e, obj, nt = dp.estep(sents, freqs, mode=S.SPM_ESTEP_FAST)
    assert nt == nt_ref
    # fp64 accumulation vs the reference's float buckets (SURVEY §8a E1:
    # up to 1.5e-4 relative at T=1).
    rel = _check_close(e, e_ref)
    assert rel < 1e-3, rel
    assert abs(obj - obj_ref) <= 1e-4 * abs(obj_ref)


@pytest.mark.parametrize("forward", FORWARDS)
@pytest.mark.parametrize("threads", [1, 16])
def test_estep_botchan_pieces_general_path(threads, forward):
    """Real text (botchan, nfkc-normalized) + the test_model's pieces; sentences
    with near-ties or odd bytes exercise the general kernel."""
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "tests", "golden", "test_model.model"))
    mb = open(os.path.join(ROOT, "tests", "golden", "test_model.model"), "rb").read()
    lines = O.read_lines_binary(os.path.join(ROOT, "tests", "golden", "botchan.txt"))
    sents = [s for s in O.OracleModel(mb).normalize(lines) if s]
    sents += [b"\xff\xfeabc", "é".encode() + b"\x80z", b"a" * 300, b"\xc3a\x80\x80b", b"ab\xe2\x96"]
    freqs = np.arange(len(sents)) % 5 + 1
    _assert_exact(sents, freqs, pieces, scores, threads, forward)


@pytest.mark.parametrize("forward", FORWARDS)
@pytest.mark.parametrize("mode", [S.SPM_ESTEP_PARITY, S.SPM_ESTEP_FAST])
def test_populate_marginal_known_answer(mode, forward):
    """LatticeTest.PopulateMarginalTest (unigram_model_test.cc:271-315) through
    spm_hip_estep: marginals and log Z within the reference's 1e-3; PARITY is
    also bit-equal to the oracle."""
    pieces, scores, sent, marg, logz, ntok = KA.populate_marginal_case()
    sc = np.array(scores, dtype=np.float32)
    dp = S.DevicePieces(pieces, sc)
    dp.set_forward(forward)
    e, obj, nt = dp.estep([sent], np.ones(1, dtype=np.int64), mode=mode, threads=1)
    assert np.allclose(e, marg, atol=1e-3), (e, marg)
    assert abs(-obj - logz) < 1e-3
    assert nt == ntok
    if mode == S.SPM_ESTEP_PARITY:
        _assert_exact([sent], np.ones(1, dtype=np.int64), pieces, sc, 1, forward)


def _long_piece_set(min_chars, seed):
    """The 32k model's pieces plus long pieces cut from the corpus itself (so
    they match), every one at least `min_chars` chars."""
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    short, freqs = _corpus(9000, seed)
    sents = [short[3 * k] + short[3 * k + 1] + short[3 * k + 2] for k in range(3000)]  # ~80 chars
    freqs = freqs[:3000]
    have = set(pieces)
    extra = []
    for s in sents:
        t = s.decode()
        if len(t) >= min_chars + 2:
            w = t[1:min_chars + 2].encode()
            if w not in have:
                have.add(w)
                extra.append(w)
        if len(extra) == 200:
            break
    assert len(extra) > 20
    rng = np.random.default_rng(seed)
    xs = (scores.min() + rng.random(len(extra)) * 4).astype(np.float32)
    return pieces + extra, np.concatenate([scores, xs]), sents, freqs


@pytest.mark.parametrize("threads", [1, 8])
def test_estep_parity_long_pieces(threads):
    """Pieces of 32+ chars (TrainerSpec allows max_sentencepiece_length up to
    512, trainer_interface.cc:74): no register ring, every sentence runs the
    general kernel after the node-count pre-pass; PARITY stays bit-exact."""
    pieces, scores, sents, freqs = _long_piece_set(40, 11)
    _assert_exact(sents, freqs, pieces, scores, threads)


def test_estep_parity_long_multibyte_walks():
    """Pieces of 22-31 CJK chars (66-93 bytes): the W = 32 ring's trie walks go
    past the 64-byte char-end mask and must take the general kernel."""
    rng = np.random.default_rng(3)
    han = [chr(0x4E00 + k) for k in range(40)]
    base = ["".join(rng.choice(han, size=int(rng.integers(22, 32)))) for _ in range(12)]
    pieces = sorted(set(han + base + ["▁"]), key=lambda x: (len(x), x))
    scores = np.array([-1.0 - 0.01 * len(p) - 0.001 * k for k, p in enumerate(pieces)], dtype=np.float32)
    sents = []
    for k in range(3000):
        parts = ["▁"] + [base[int(rng.integers(0, len(base)))] if rng.random() < 0.5 else
                         "".join(rng.choice(han, size=int(rng.integers(1, 6)))) for _ in range(3)]
        sents.append("".join(parts).encode())
    freqs = np.arange(len(sents)) % 3 + 1
    for T in (1, 8):
        _assert_exact(sents, freqs, [p.encode() for p in pieces], scores, T)


@pytest.mark.parametrize("forward", FORWARDS)
@pytest.mark.parametrize("threads", [1, 8])
def test_estep_parity_unk_id_collision(threads, forward):
    """TrainerModel's unk id is 0, the id of the first piece (unigram_model_trainer.h:39-89).
    With a multi-char piece 0 ("ab") and no single-char piece for 'a', a lattice position
    holds both the trie node of piece 0 and the UNK node (id 0 too): their two records share
    one key, so they must reach the fold in begin_nodes order (trie nodes, then UNK).  The
    lagged PARITY backward kernel writes a position's records from the block's end and
    reserves the UNK slot last; this pins that order bit-exactly."""
    rng = np.random.default_rng(21)
    pieces = [p.encode() for p in ["ab", "b", "c", "bc", "abc", "cab", "▁", "▁ab", "ca"]]
    scores = np.array([-1.5, -2.0, -2.5, -3.0, -3.5, -4.0, -1.0, -2.25, -2.75], dtype=np.float32)
    sents, freqs = [], []
    for _ in range(20000):
        L = int(rng.integers(1, 30))
        sents.append(("▁" + "".join("abc"[int(x)] for x in rng.integers(0, 3, L))).encode())
        freqs.append(int(rng.integers(1, 4)))
    _assert_exact(sents, np.array(freqs), pieces, scores, threads, forward)


def test_estep_parity_deferred_folds_across_calls():
    """SPM_ESTEP_DEFER_FOLD: a corpus fed as several accumulate calls (the
    bench's resident-buffer chunks, dist_estep.DeviceEStep) with each call's
    last fold left running beside the next call's walks, completed by
    spm_hip_estep_sync / finalize, equals the oracle bit for bit.  Chunks of
    > 4M sentences would exercise the in-call overlap too; here each call is
    smaller than one fold chunk, so every fold overlaps across calls."""
    import torch
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    sents, freqs = _corpus(40000, 9)
    T = 8
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, T)
    dp = S.DevicePieces(pieces, scores)
    dev = torch.device("cuda", 0)
    V = dp.V
    acc = torch.zeros(T * V, dtype=torch.float32, device=dev)
    acc_obj = torch.zeros(T, dtype=torch.float32, device=dev)
    ntok = torch.zeros(T, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    n = len(sents)
    cuts = [0, 7000, 7001, 19000, 31000, n]  # calls of 7000, 1, 11999, 12000, 9000 sentences
    keep = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        buf, off = S.to_csr(sents[a:b])
        db = torch.from_numpy(buf).to(dev)
        do = torch.from_numpy(off.view(np.int64)).to(dev)
        df = torch.from_numpy(np.ascontiguousarray(freqs[a:b], dtype=np.int64)).to(dev)
        keep += [db, do, df]  # inputs stay alive until the folds are synced
        dp.accumulate_device(db.data_ptr(), do.data_ptr(), df.data_ptr(), b - a, int(np.sum(freqs)),
                             S.SPM_ESTEP_PARITY, T, a, 1, acc.data_ptr(), acc_obj.data_ptr(), ntok.data_ptr(),
                             stream, defer=True)
    dp.sync_device(stream)
    e = torch.empty(V, dtype=torch.float32, device=dev)
    o = torch.empty(1, dtype=torch.float32, device=dev)
    nt = torch.empty(1, dtype=torch.int64, device=dev)
    dp.finalize_device(S.SPM_ESTEP_PARITY, T, acc.data_ptr(), acc_obj.data_ptr(), ntok.data_ptr(),
                       e.data_ptr(), o.data_ptr(), nt.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    e = e.cpu().numpy()
    bad = np.nonzero(e.view(np.uint32) != e_ref.view(np.uint32))[0]
    assert len(bad) == 0, ("inexact pieces", len(bad))
    assert np.float32(o.item()).view(np.uint32) == np.float32(obj_ref).view(np.uint32)
    assert int(nt.item()) == nt_ref
    dp.close()


@pytest.mark.parametrize("forward", [0, 1])
@pytest.mark.parametrize("neg", [False, True])
def test_estep_parity_record_drop(monkeypatch, neg, forward):
    """PARITY record drop (estep_threshold_kernel): with chunks of 64k
    sentences, every chunk after the first reads lower bounds of its
    accumulators and does not write records below a quarter ulp of them.
    The result stays bit-exact, and most records are dropped.  A negative
    sentence freq (contributions that could lower an accumulator) turns the
    drop off for the rest of the piece set's life: the chunks before it
    dropped soundly, the ones after keep every record.  forward=1 (the byte
    kernel's forward pass) also takes the tile-transposed alpha and records
    (EArgs::AT / RT); the long sentences among the short ones go past their
    64 rows of alpha and 32 kept records per lane into the range layout."""
    monkeypatch.setenv("SPM_HIP_ESTEP_CHUNK", "65536")
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    sents, freqs = _corpus(300000, 17)
    for k in range(0, 300000, 97):  # every 97th sentence: 4-9 sentences joined (~130-300 B)
        sents[k] = b"".join(sents[k:k + 4 + k % 6])
    if neg:
        freqs = freqs.copy()
        freqs[200000] = -2
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, 16)
    dp = S.DevicePieces(pieces, scores)
    dp.set_forward(forward)
    e, obj, nt = dp.estep(sents, freqs, mode=S.SPM_ESTEP_PARITY, threads=16)
    written, kept = dp.record_stats()
    bad = np.nonzero(e.view(np.uint32) != e_ref.view(np.uint32))[0]
    assert len(bad) == 0, ("inexact pieces", len(bad))
    assert np.float32(obj).view(np.uint32) == np.float32(obj_ref).view(np.uint32)
    assert nt == nt_ref
    assert 0 < kept < written
    if not neg:
        assert kept < 0.5 * written, (kept, written)
    else:
        # the drop is off from the chunk holding the negative freq on (3 of 5 chunks)
        assert kept > 0.5 * written, (kept, written)
    dp.close()


@pytest.mark.parametrize("forward", FORWARDS)
def test_estep_set_scores_equals_fresh_pieces(forward):
    """spm_hip_pieces_set_scores (the trainer's next E-step when the M-step
    dropped no piece): an E-step under the new scores is bit-exact with the
    oracle's, after an E-step under the old ones on the same handle (work
    buffers, hot table, byte-kernel model all carried over); a wrong piece
    count is refused."""
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    sents, freqs = _corpus(30000, 11)
    rng = np.random.default_rng(3)
    new = (scores + rng.normal(0, 0.5, size=len(scores))).astype(np.float32)
    dp = S.DevicePieces(pieces, scores)
    dp.set_forward(forward)
    dp.estep(sents, freqs, mode=S.SPM_ESTEP_PARITY, threads=8)
    dp.set_scores(new)
    e, obj, nt = dp.estep(sents, freqs, mode=S.SPM_ESTEP_PARITY, threads=8)
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, new, 8)
    bad = np.nonzero(e.view(np.uint32) != e_ref.view(np.uint32))[0]
    assert len(bad) == 0, len(bad)
    assert np.float32(obj).view(np.uint32) == np.float32(obj_ref).view(np.uint32)
    assert nt == nt_ref
    fresh = S.DevicePieces(pieces, new)
    fresh.set_forward(forward)
    e2, _, _ = fresh.estep(sents, freqs, mode=S.SPM_ESTEP_FAST)
    dp_fast = dp.estep(sents, freqs, mode=S.SPM_ESTEP_FAST)[0]
    assert np.array_equal(e2.view(np.uint32), dp_fast.view(np.uint32))
    rc = S.lib().spm_hip_pieces_set_scores(dp.h, S._p(new), dp.V + 1)
    assert rc == 11  # SPM_OUT_OF_RANGE
