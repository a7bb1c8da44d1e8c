"""CPU: the oracle against the reference's own fixtures and known answers."""
import os

import numpy as np
import pytest

import known_answers as KA
import oracle_lib as O
from model_builder import CONTROL, NORMAL, UNKNOWN, model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _gold(name):
    return [list(map(int, l.split())) for l in open(os.path.join(GOLD, name)).read().split("\n")[:-1]]


@pytest.mark.parametrize("model_name,text,golden", [
    ("test_model.model", "botchan.txt", "botchan_test_model.ids"),
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt", "wagahaiwa_test_ja_model.ids"),
    ("botchan_bpe1k.model", "botchan.txt", "botchan_bpe1k.ids"),
])
def test_oracle_matches_golden_ids(model_name, text, golden):
    """spm_encode --output_format=id (sha256 of the botchan output equals the
    one the survey measured with the real reference build: f8c9f177...)."""
    m = O.OracleModel(open(os.path.join(GOLD, model_name), "rb").read())
    lines = O.read_lines_binary(os.path.join(GOLD, text))
    assert m.encode_lines(lines) == _gold(golden)


@pytest.mark.parametrize("name", [c[0] for c in KA.cases()])
def test_oracle_known_answers(name):
    _, mb, exp = [c for c in KA.cases() if c[0] == name][0]
    m = O.OracleModel(mb)
    for inp, want in exp:
        buf, off = O.to_csr([KA.as_bytes(inp)])
        ids, lens, to = m.encode_normalized_csr(buf, off, with_lens=True)
        assert KA.split_pieces(inp, lens) == [KA.as_bytes(w) for w in want], inp


def test_oracle_processor_extra_options():
    """SentencePieceProcessorTest.EndToEndTest (sentencepiece_processor_test.cc:640-816)."""
    pieces = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL),
              ("a", 0.0, NORMAL), ("b", 0.3, NORMAL), ("c", 0.2, NORMAL), ("ab", 1.0, NORMAL),
              ("▁", 3.0, NORMAL)]
    m = O.OracleModel(model(pieces))
    for opt, want in [("", [7, 6, 5]), ("bos", [1, 7, 6, 5]), ("eos", [7, 6, 5, 2]),
                      ("reverse", [5, 6, 7]), ("bos:eos", [1, 7, 6, 5, 2]),
                      ("reverse:bos:eos", [1, 5, 6, 7, 2]), ("bos:eos:reverse", [2, 5, 6, 7, 1])]:
        m.set_extra_options(opt)
        assert m.encode_lines([b"abc"]) == [want], opt


def test_oracle_unk_merge():
    """Consecutive UNKNOWN pieces become one id (sentencepiece_processor.cc:525-529)."""
    pieces = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL),
              ("a", -1.0, NORMAL), ("▁", -1.0, NORMAL)]
    m = O.OracleModel(model(pieces))
    assert m.encode_lines([b"xyzaxy"]) == [[4, 0, 3, 0]]


def test_oracle_estep_thread_buckets_differ():
    """RunEStep's result depends on num_threads (float bucket order)."""
    import model_reader
    import synth
    mb = open(os.path.join(GOLD, "test_model.model"), "rb").read()
    pcs = [(p, s) for p, s, t in model_reader.read_pieces(mb) if t == 1]
    pieces = [p for p, _ in pcs]
    scores = np.array([s for _, s in pcs], dtype=np.float32)
    buf, off = synth.normalized(20000, seed=1)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(20000)]
    f = np.ones(20000, dtype=np.int64)
    e1, o1, n1 = O.estep(sents, f, pieces, scores, 1)
    e8, o8, n8 = O.estep(sents, f, pieces, scores, 8)
    assert n1 == n8
    nz = e1 != 0
    rel = np.abs(e1 - e8)[nz] / e1[nz]
    assert rel.max() < 1e-3 and np.any(e1 != e8)


def test_oracle_populate_marginal_known_answer():
    """LatticeTest.PopulateMarginalTest (unigram_model_test.cc:271-315) through
    the oracle's RunEStep: expected[id] = the node marginals (±1e-3 as the
    reference test), obj = -log Z, ntok = the Viterbi size."""
    pieces, scores, sent, marg, logz, ntok = KA.populate_marginal_case()
    for T in (1, 8):
        e, obj, nt = O.estep([sent], np.ones(1, dtype=np.int64), pieces,
                             np.array(scores, dtype=np.float32), T)
        assert np.allclose(e, marg, atol=1e-3), (e, marg)
        assert abs(-obj - logz) < 1e-3
        assert nt == ntok


def test_oracle_estep_cyclic_equals_repeated_corpus():
    """oracle_estep_cyclic (sentence g = buffer[g mod n], what bench.py's
    full-size c4 PARITY check runs) equals oracle_estep on the explicitly
    repeated corpus, bit for bit, for a total that is not a multiple of n."""
    import model_reader
    import synth
    pcs = [(p, s) for p, s, t in model_reader.read_pieces(
        open(os.path.join(ROOT, "data", "synth32k_unigram.model"), "rb").read()) if t == 1]
    pieces = [p for p, _ in pcs]
    scores = np.array([s for _, s in pcs], dtype=np.float32)
    buf, off = synth.normalized(1500, seed=3)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(1500)]
    freqs = np.arange(1500) % 3 + 1
    total = 3 * 1500 + 700
    rep = [sents[g % 1500] for g in range(total)]
    rfreq = np.array([freqs[g % 1500] for g in range(total)])
    e0, o0, n0 = O.estep(rep, rfreq, pieces, scores, 16)
    e1, o1, n1 = O.estep_cyclic_csr(buf, off, freqs, total, pieces, scores, 16)
    assert np.array_equal(e0.view(np.uint32), e1.view(np.uint32))
    assert np.float32(o0).view(np.uint32) == np.float32(o1).view(np.uint32) and n0 == n1
