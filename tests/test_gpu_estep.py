"""GPU parity of the unigram trainer E-step (RunEStep) vs the CPU oracle."""
import os

import numpy as np
import pytest

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


def _check_close(got, ref, rtol):
    nz = ref != 0
    rel = np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])
    assert np.all(got[~nz] == 0)
    return float(rel.max()) if rel.size else 0.0


@pytest.mark.parametrize("threads", [1, 8, 16])
def test_estep_parity_mode(threads):
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    sents, freqs = _corpus(60000, 5)
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, threads)
    dp = S.DevicePieces(pieces, scores)
    e, obj, nt = dp.estep(sents, freqs, mode=S.SPM_ESTEP_PARITY, threads=threads)
    assert nt == nt_ref
    exact = np.mean(e == e_ref)
    rel = _check_close(e, e_ref, 1e-6)
    # Bit-exact apart from rare device-vs-glibc exp/log ulp differences.
    assert exact > 0.999 and rel < 1e-5, (exact, rel)
    assert abs(obj - obj_ref) <= 1e-6 * abs(obj_ref)


def test_estep_fast_mode():
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "data", "synth32k_unigram.model"))
    sents, freqs = _corpus(60000, 6)
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, 1)
    dp = S.DevicePieces(pieces, scores)
    e, obj, nt = dp.estep(sents, freqs, mode=S.SPM_ESTEP_FAST)
    assert nt == nt_ref
    # fp64 accumulation vs the reference's float buckets (SURVEY §8a E1:
    # up to 1.5e-4 relative at T=1).
    rel = _check_close(e, e_ref, 1e-3)
    assert rel < 1e-3, rel
    assert abs(obj - obj_ref) <= 1e-4 * abs(obj_ref)


def test_estep_botchan_pieces_general_path():
    """Real text (botchan, nfkc-normalized) + the test_model's pieces; sentences
    with near-ties or odd bytes exercise the general kernel."""
    pieces, scores = _pieces_from_model(os.path.join(ROOT, "tests", "golden", "test_model.model"))
    mb = open(os.path.join(ROOT, "tests", "golden", "test_model.model"), "rb").read()
    lines = O.read_lines_binary(os.path.join(ROOT, "tests", "golden", "botchan.txt"))
    sents = [s for s in O.OracleModel(mb).normalize(lines) if s]
    sents += [b"\xff\xfeabc", "é".encode() + b"\x80z", b"a" * 300]
    freqs = np.arange(len(sents)) % 5 + 1
    for threads in (1, 16):
        e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, threads)
        dp = S.DevicePieces(pieces, scores)
        e, obj, nt = dp.estep(sents, freqs, mode=S.SPM_ESTEP_PARITY, threads=threads)
        assert nt == nt_ref
        assert np.mean(e == e_ref) > 0.99
        assert _check_close(e, e_ref, 1e-5) < 1e-5
