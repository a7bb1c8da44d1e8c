"""GPU: SentencePieceProcessor::Encode(input, SentencePieceText*) on the
device (spm_hip_encode_spt: Normalize with norm_to_orig, Encode,
PopulateSentencePieceText sentencepiece_processor.cc:488-551 and
ApplyExtraOptions :945-979) against the oracle's restatement: every piece's
id, piece string, surface and begin/end byte offsets, including merged
UNKNOWN runs, the NormalizerSpec switches and the extra options."""
import os

import pytest

import oracle_lib as O
import synth
from model_builder import CONTROL, NORMAL, UNKNOWN, USER_DEFINED, model
from model_reader import charsmap
from test_gpu_normalize import EDGE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
pytestmark = pytest.mark.gpu


def _check(mb, lines, opts=""):
    import spm_amd
    dm = spm_amd.DeviceModel(mb)
    got = dm.encode_spt_device(lines, opts)
    om = O.OracleModel(mb)
    om.set_extra_options(opts)
    want = om.encode_spt(lines)
    bad = []
    for i, (g, w) in enumerate(zip(got, want)):
        ok = len(g) == len(w) and all(
            gi[0] == wi[0] and (gi[1] is None or gi[1] == wi[1]) and gi[2:] == wi[2:] for gi, wi in zip(g, w))
        if not ok:
            bad.append(i)
    assert not bad, [(lines[i][:40], got[i][:4], want[i][:4]) for i in bad[:3]]
    return got


@pytest.mark.parametrize("model_name,text", [
    ("test_model.model", "botchan.txt"),
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt"),
    ("botchan_bpe1k.model", "botchan.txt"),
])
@pytest.mark.parametrize("opts", ["", "bos:eos", "reverse", "bos:reverse:eos"])
def test_encode_spt_golden(model_name, text, opts):
    mb = open(os.path.join(GOLD, model_name), "rb").read()
    _check(mb, O.read_lines_binary(os.path.join(GOLD, text)) + EDGE, opts)


def test_encode_spt_synthetic():
    mb = open(os.path.join(ROOT, "data", "synth32k_unigram.model"), "rb").read()
    got = _check(mb, synth.lines(50_000, seed=21) + EDGE)
    # surfaces tile the line: each piece starts where the previous one ended
    for g in got[:1000]:
        assert all(a[4] == b[3] for a, b in zip(g, g[1:]))


def test_encode_spt_unknown_runs():
    """Runs of UNKNOWN pieces merge into one piece whose surface spans the
    run (sentencepiece_processor.cc:525-529)."""
    pieces = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL),
              ("▁", -1.0, NORMAL), ("a", -1.0, NORMAL), ("b", -2.0, NORMAL), ("▁a", -0.5, NORMAL),
              ("<tag>", 0.0, USER_DEFINED)]
    mb = model(pieces)
    lines = [b"a xyz b", "ａ漢字ｂ  ｃ".encode(), b"<tag>qq<tag>", b"  zz  ", b"q", b"", b"a\xffb"]
    got = _check(mb, lines)
    assert any(len(p[2]) > 1 and p[0] == 0 for g in got for p in g)


@pytest.mark.parametrize("opts", [
    dict(add_dummy_prefix=False),
    dict(remove_extra_whitespaces=False),
    dict(escape_whitespaces=False),
    dict(treat_ws_as_suffix=True),
    dict(treat_ws_as_suffix=True, remove_extra_whitespaces=False),
])
def test_encode_spt_spec_switches(opts):
    cm = charsmap(open(os.path.join(GOLD, "test_model.model"), "rb").read())
    pieces = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL),
              ("a", -1.0, NORMAL), ("▁", -2.0, NORMAL), (" ", -2.0, NORMAL), ("b", -1.5, NORMAL),
              ("<user>", 0.0, USER_DEFINED)]
    mb = model(pieces, charsmap=cm, **opts)
    _check(mb, EDGE + [b"  a  b ", "ab ｂａ <user>a".encode(), b" a\tb "], "bos:eos")


def test_normalize_full_test_reference_vectors():
    """NormalizeFullTest (normalizer_test.cc:321-401): the reference's exact
    normalized strings and n2i vectors through the device normalizer
    (spm_hip_normalize_batch_device_align)."""
    import spm_amd
    import spt_known_answers as KA
    dm = spm_amd.DeviceModel(KA.normalizer_model())
    got = dm.normalize_align_device([i.encode() for i, _, _ in KA.NORMALIZE_FULL])
    for (inp, want, n2i), (norm, a) in zip(KA.NORMALIZE_FULL, got):
        assert norm == want.encode(), inp
        assert a == n2i, inp


def test_encode_test_reference_spt():
    """SentencepieceProcessorTest.EncodeTest (sentencepiece_processor_test.cc:
    129-240): piece / surface / id / begin / end of Encode("ABC DEF") through
    spm_hip_encode_spt, including the merged UNKNOWN run "EF" (tests/
    spt_known_answers.py explains the model stand-ins for the MockModel)."""
    import spm_amd
    import spt_known_answers as KA
    for name, pieces, rows in KA.ENCODE_CASES:
        dm = spm_amd.DeviceModel(KA.encode_model(pieces))
        got = dm.encode_spt_device([KA.ENCODE_INPUT], "eos")[0]
        want = [(i, p.encode(), s.encode(), b, e) for i, p, s, b, e in rows]
        # The device returns the piece as a view of the normalized line; the
        # eos extra carries None (its piece is IdToPiece(id)).
        assert [(g[0], g[2], g[3], g[4]) for g in got] == [(w[0], w[2], w[3], w[4]) for w in want], name
        assert [g[1] for g in got[:-1]] == [w[1] for w in want[:-1]] and got[-1][1] is None, name
