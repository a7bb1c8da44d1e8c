"""CPU: the C-ABI library loads, exports what include/spm_hip.h declares, and
its host-side logic (proto parsing, InitializePieces checks, trie build,
normalizer) matches the oracle — no GPU calls."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_lib as O
import synth
from model_builder import CONTROL, NORMAL, UNKNOWN, model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def S():
    import spm_amd
    if not os.path.exists(spm_amd.LIB_PATH):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "sentencepiece-comments_amd")])
    spm_amd.lib()
    return spm_amd


def test_exports_match_header(S):
    hdr = open(os.path.join(ROOT, "include", "spm_hip.h")).read()
    declared = set(re.findall(r"\b(spm_hip_\w+)\s*\(", hdr))
    assert declared == set(S.EXPORTED)
    L = S.lib()
    for name in declared:
        assert hasattr(L, name), name


@pytest.mark.parametrize("name,kind,pieces,chars", [
    ("tests/golden/test_model.model", 1, 1000, 13),
    ("tests/golden/test_ja_model.model", 1, 8000, 9),
    ("data/synth32k_unigram.model", 1, 32000, 11),
    ("data/synth32k_bpe.model", 2, 32000, 0),
])
def test_host_only_load(S, name, kind, pieces, chars):
    d = S.DeviceModel(open(os.path.join(ROOT, name), "rb").read(), host_only=True)
    inf = d.info()
    assert (inf.model_type, inf.piece_size, inf.max_piece_chars) == (kind, pieces, chars)
    assert inf.unk_id == 0
    # encode on a host-only handle fails loudly (FAILED_PRECONDITION)
    with pytest.raises(S.SpmError) as e:
        d.encode_normalized([b"abc"])
    assert e.value.code == 9


def test_load_errors(S):
    # Status codes follow util::error::Code; InitializePieces checks
    # (model_interface.cc:101-144) map to INTERNAL (13).
    base = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL)]
    bad = {
        "garbage": b"\xff\xff\xff\xff",
        "no_unk": model([("a", 0.0, NORMAL)]),
        "dup": model(base + [("a", 0.0, NORMAL), ("a", 0.0, NORMAL)]),
        "two_unk": model(base + [("<unk2>", 0.0, UNKNOWN)]),
        "empty_piece": model(base + [("", 0.0, NORMAL)]),
    }
    for k, mb in bad.items():
        with pytest.raises(S.SpmError) as e:
            S.DeviceModel(mb, host_only=True)
        assert e.value.code == 13, k


@pytest.mark.parametrize("model_name,text", [
    ("test_model.model", "botchan.txt"),
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt"),
])
def test_normalizer_matches_oracle(S, model_name, text):
    mb = open(os.path.join(GOLD, model_name), "rb").read()
    lines = O.read_lines_binary(os.path.join(GOLD, text))
    lines += [b"", b"   ", b"  a  b  ", b"\xff\xfe", "ｱｲｳ①Ⅷ".encode(), b"\t\r\n x"]
    d = S.DeviceModel(mb, host_only=True)
    assert d.normalize(lines) == O.OracleModel(mb).normalize(lines)


def test_synth_normalized_claim(S):
    """tools/synth.py emits exactly what the model's normalizer produces."""
    mb = open(os.path.join(ROOT, "data", "synth32k_unigram.model"), "rb").read()
    d = S.DeviceModel(mb, host_only=True)
    raw = synth.lines(5000, seed=9)
    nb, no = synth.normalized(5000, seed=9)
    b = nb.tobytes()
    want = [b[int(no[i]):int(no[i + 1])] for i in range(5000)]
    assert d.normalize(raw) == want
