"""GPU: Normalizer::Normalize on the device (spm_hip_normalize_batch_device)
is byte-identical to the oracle's restatement (normalizer.cc:88-300) for the
reference's own models (nfkc / nmt_nfkc charsmaps), the NormalizerSpec
switches, user-defined symbols and edge cases."""
import os

import pytest

import oracle_lib as O
import synth
from model_builder import CONTROL, NORMAL, UNKNOWN, USER_DEFINED, model
from model_reader import charsmap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
pytestmark = pytest.mark.gpu

EDGE = [b"", b" ", b"   ", b"  a  b  ", b"\xff\xfe", "ｱｲｳ①Ⅷ".encode(), b"\t\r\n x", b"a\xe2\x96\x81",
        "▁▁a▁▁".encode(), "  ▁ x ▁ ".encode(), b"\xe2\x96", b"x\x00y", "ﷺ ﬁ ㍿".encode(),
        "<s>a</s> <user>b".encode(), "　全角　スペース　".encode(), b"a" * 5000]


def _check(mb, lines):
    import spm_amd
    dm = spm_amd.DeviceModel(mb)
    got = dm.normalize_device(lines)
    want = O.OracleModel(mb).normalize(lines)
    bad = [i for i in range(len(lines)) if got[i] != want[i]]
    assert not bad, [(lines[i][:60], got[i][:60], want[i][:60]) for i in bad[:5]]
    _check_align(dm, mb, lines)


def _check_align(dm, mb, lines):
    """norm_to_orig (spm_hip_normalize_batch_device_align) equals the
    reference's vector (normalizer.cc:88-211) wherever the reference builds
    one; where it returns early with an empty vector (empty or all-whitespace
    line) the device's single entry is the consumed byte count."""
    got = dm.normalize_align_device(lines)
    want = O.OracleModel(mb).normalize_align(lines)
    bad = []
    for i, ((gn, ga), (wn, wa)) in enumerate(zip(got, want)):
        assert len(ga) == len(gn) + 1
        if gn != wn or (wa and ga != wa) or (not wa and (gn or ga[0] > len(lines[i]))):
            bad.append(i)
    assert not bad, [(lines[i][:40], got[i][1][:20], want[i][1][:20]) for i in bad[:5]]


@pytest.mark.parametrize("model_name,text", [
    ("test_model.model", "botchan.txt"),
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt"),
    ("test_model.model", "wagahaiwa_nekodearu.txt"),
])
def test_device_normalizer_golden(model_name, text):
    mb = open(os.path.join(GOLD, model_name), "rb").read()
    _check(mb, O.read_lines_binary(os.path.join(GOLD, text)) + EDGE)


def test_device_normalizer_synthetic_nmt_nfkc():
    mb = open(os.path.join(ROOT, "data", "synth32k_unigram.model"), "rb").read()
    _check(mb, synth.lines(200_000, seed=5) + EDGE)


@pytest.mark.parametrize("opts", [
    dict(add_dummy_prefix=False),
    dict(remove_extra_whitespaces=False),
    dict(escape_whitespaces=False),
    dict(treat_ws_as_suffix=True),
    dict(treat_ws_as_suffix=True, remove_extra_whitespaces=False),
    dict(add_dummy_prefix=False, remove_extra_whitespaces=False, escape_whitespaces=False),
])
@pytest.mark.parametrize("rule", ["identity", "nfkc"])
def test_device_normalizer_spec_switches(opts, rule):
    cm = b"" if rule == "identity" else charsmap(open(os.path.join(GOLD, "test_model.model"), "rb").read())
    pieces = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL),
              ("a", -1.0, NORMAL), ("<user>", 0.0, USER_DEFINED), ("▁x y", 0.0, USER_DEFINED)]
    mb = model(pieces, charsmap=cm, **opts)
    lines = O.read_lines_binary(os.path.join(GOLD, "botchan.txt"))[:500] + EDGE + \
        [b" <user> a<user><user> ", "x y ▁x y".encode()]
    _check(mb, lines)
