"""GPU parity: the HIP encode path (through the C-ABI) vs the CPU oracle.

Bit-exact token ids and piece byte lengths on the same normalized inputs.
Sizes are chosen so the oracle finishes in seconds.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
import spm_amd as S
import model_reader
import synth
from model_builder import BPE, CONTROL, NORMAL, UNIGRAM, UNUSED, USER_DEFINED, base_pieces, model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(ROOT, "data")

pytestmark = pytest.mark.gpu


def _read(p):
    return open(p, "rb").read()


def _compare(mb, sentences, force_general=False, dm=None):
    """Encodes normalized sentences on the GPU and with the oracle; asserts equal."""
    dm = dm or S.DeviceModel(mb)
    dm.set_force_general(force_general)
    buf, off = S.to_csr(sentences)
    ids, lens, to = dm.encode_csr_host(buf, off, with_lens=True)
    om = O.OracleModel(mb)
    oids, olens, oto = om.encode_normalized_csr(buf, off, threads=8, with_lens=True)
    assert np.array_equal(to, oto), "token counts differ"
    bad = np.nonzero(ids != oids)[0]
    assert bad.size == 0, "first mismatch at token %d" % bad[0]
    assert np.array_equal(lens, olens)
    return dm.stats()


def _golden_ids(name):
    return [list(map(int, l.split())) for l in open(os.path.join(GOLD, name)).read().split("\n")[:-1]]


def _merge_unk(ids, lens, unk_ids):
    # PopulateSentencePieceText (sentencepiece_processor.cc:488-551): a run of
    # UNKNOWN pieces becomes one piece.
    out = []
    prev_unk = False
    for i in ids:
        u = i in unk_ids
        if not (prev_unk and u):
            out.append(i)
        prev_unk = u
    return out


@pytest.mark.parametrize("model_name,text,golden", [
    ("test_model.model", "botchan.txt", "botchan_test_model.ids"),
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt", "wagahaiwa_test_ja_model.ids"),
    ("botchan_bpe1k.model", "botchan.txt", "botchan_bpe1k.ids"),
])
def test_end_to_end_golden(model_name, text, golden):
    """Config c1: spm_encode --output_format=id ids == golden fixture."""
    _golden_check(model_name, text, golden)


def test_end_to_end_golden_ja_char_kernel(monkeypatch):
    """The ja model takes the wide-char kernel; SPM_HIP_NO_WIDE keeps it on the
    char kernel (W = 32): both match the reference's golden ids."""
    monkeypatch.setenv("SPM_HIP_NO_WIDE", "1")
    assert _golden_check("test_ja_model.model", "wagahaiwa_nekodearu.txt", "wagahaiwa_test_ja_model.ids") == (2, 32)


def _golden_check(model_name, text, golden):
    mb = _read(os.path.join(GOLD, model_name))
    lines = O.read_lines_binary(os.path.join(GOLD, text))
    dm = S.DeviceModel(mb)
    norm = dm.normalize(lines)
    buf, off = S.to_csr(norm)
    ids, to = dm.encode_csr_host(buf, off)
    gold = _golden_ids(golden)
    unk = {dm.info().unk_id}
    bad = 0
    for i in range(len(lines)):
        got = _merge_unk(ids[int(to[i]):int(to[i + 1])].tolist(), None, unk)
        bad += got != gold[i]
    assert bad == 0
    if model_name == "test_ja_model.model" and not os.environ.get("SPM_HIP_NO_WIDE"):
        assert dm.info().fast_variant == 3  # the wide-char kernel
    return dm.info().fast_variant, dm.info().ring_width


@pytest.mark.parametrize("model_name,text", [
    ("test_model.model", "botchan.txt"),
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt"),
    ("botchan_bpe1k.model", "botchan.txt"),
])
@pytest.mark.parametrize("force_general", [False, True])
def test_model_encode_vs_oracle(model_name, text, force_general):
    mb = _read(os.path.join(GOLD, model_name))
    lines = O.read_lines_binary(os.path.join(GOLD, text))
    norm = O.OracleModel(mb).normalize(lines)
    _compare(mb, norm, force_general)


@pytest.mark.parametrize("kind", ["unigram", "bpe"])
def test_synth_32k(kind):
    """c2/c3 models on 200k synthetic sentences."""
    mb = _read(os.path.join(DATA, "synth32k_%s.model" % kind))
    buf, off = synth.normalized(200000, seed=7)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    st = _compare(mb, sents)
    assert st.general_path < 2000


@pytest.mark.parametrize("kind", ["unigram", "bpe"])
def test_synth_32k_general_path(kind):
    mb = _read(os.path.join(DATA, "synth32k_%s.model" % kind))
    buf, off = synth.normalized(5000, seed=11)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
    _compare(mb, sents, force_general=True)


def _synth_model(extra_piece_bytes=0):
    """The c2 32k unigram model, optionally with one extra NORMAL piece of
    extra_piece_bytes bytes ("▁q…q"), which moves the model to another
    encode kernel: < 16 bytes byte kernel, < 64 char kernel, else general.
    A negative value -k adds "▁" + "é" * k instead (2-byte chars: 3 + 2k
    bytes in k + 1 chars), the wide-char kernel's kind of model."""
    mb = _read(os.path.join(DATA, "synth32k_unigram.model"))
    if not extra_piece_bytes:
        return mb, []
    pcs = [(p, s, t) for p, s, t in model_reader.read_pieces(mb)]
    if extra_piece_bytes < 0:
        longp = ("▁" + "é" * -extra_piece_bytes).encode()
        pcs.append((longp, -30.0, NORMAL))
        pcs.append(("é".encode(), -12.0, NORMAL))
        return model(pcs, UNIGRAM), [longp, longp + b"zz", b"q" + longp, longp[:-1], "é".encode() * 40]
    longp = "▁".encode() + b"q" * (extra_piece_bytes - 3)
    pcs.append((longp, -30.0, NORMAL))
    return model(pcs, UNIGRAM), [longp, longp + b"zz", b"q" + longp]


# Long LAST sentence: its EOS back-pointer sits one past the batch's last
# byte, beyond the 64-byte LDS window (the round-2 hang's exact position).
_LONG_LAST = "▁".encode() + b"abcdefgh" * 12


@pytest.mark.parametrize("extra,kernel,ring", [(0, 1, 16), (20, 2, 32), (40, 2, 64), (70, 0, 0), (-9, 3, 16),
                                               (-14, 3, 16)])
def test_unigram_encode_kernels(extra, kernel, ring):
    """Every unigram encode kernel that ships (spm_hip_model_info.fast_variant:
    1 byte kernel, 2 char kernel W = 32/64, 3 wide-char kernel (16-char ring,
    pieces of 16-63 bytes in < 16 chars), 0 general only), chosen by the
    model's longest piece, bit-exact vs the oracle on synthetic + edge
    sentences, with a > 64-byte sentence last in the batch."""
    mb, extra_sents = _synth_model(extra)
    dm = S.DeviceModel(mb)
    inf = dm.info()
    assert (inf.fast_variant, inf.ring_width) == (kernel, ring)
    buf, off = synth.normalized(30000, seed=13)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)] + _edge_sentences() + extra_sents
    _compare(mb, sents + [_LONG_LAST], dm=dm)


@pytest.mark.parametrize("extra", [0, 20, -9])
def test_unigram_near_tie_stress(extra):
    """Near-tie stress: every multi-char piece scores one float ulp below the
    float sum of its first char and the rest, so at most end positions a
    later-inserted path beats an earlier one by about an ulp.  The fast
    kernel's near-tie entries fill up (byte kernel 2 per sentence, char
    kernel 4) and overflowing / 3-deep sentences take the general kernel
    through the device-count path and the fix-up chain; ids and lengths stay
    bit-exact."""
    rng = np.random.default_rng(5)
    alpha = "abcdef"
    f32 = np.float32
    sc = {"▁": f32(-1.0)}
    for c in alpha:
        sc[c] = f32(-rng.uniform(1.0, 3.0))
    for L in (2, 3, 4):
        for _ in range(60):
            w = "".join(alpha[int(x)] for x in rng.integers(0, len(alpha), L))
            if w in sc or w[1:] not in sc:
                continue
            tot = f32(sc[w[0]] + sc[w[1:]])
            sc[w] = np.nextafter(tot, f32(-np.inf)) if rng.random() < 0.7 else tot
    pieces = base_pieces() + [(w, float(v), NORMAL) for w, v in sc.items()]
    if extra > 0:
        pieces.append(("▁" + "q" * (extra - 3), -30.0, NORMAL))
    elif extra < 0:
        pieces.append(("▁" + "é" * -extra, -30.0, NORMAL))
    mb = model(pieces, UNIGRAM)
    sents = []
    for _ in range(20000):
        L = int(rng.integers(0, 40))
        sents.append(("▁" + "".join(alpha[int(x)] for x in rng.integers(0, len(alpha), L))).encode())
    dm = S.DeviceModel(mb)
    assert dm.info().fast_variant == (2 if extra > 0 else 3 if extra < 0 else 1)
    st = _compare(mb, sents + [_LONG_LAST], dm=dm)
    assert st.general_path > 0  # the overflow route was exercised


@pytest.mark.parametrize("extra", [0, 20, -9])
@pytest.mark.parametrize("where", ["lds", "global"])
def test_corrupt_back_pointer_takes_general_path(extra, where):
    """Debug knob: the fast kernel zeroes one sentence's EOS back-pointer
    after its forward pass (in LDS for a short sentence, in the global
    scratch for the > 64-byte last sentence).  The backtrace's bound check
    flags the sentence instead of looping; it is re-run by the general
    kernel and the batch stays bit-exact."""
    mb, _ = _synth_model(extra)
    buf, off = synth.normalized(3000, seed=21)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)] + [_LONG_LAST]
    victim = 1500 if where == "lds" else len(sents) - 1
    dm = S.DeviceModel(mb)
    dm.set_debug_corrupt_bp(victim)
    st = _compare(mb, sents, dm=dm)
    assert st.general_path >= 1


def _edge_sentences():
    ws = "▁".encode()
    return [
        b"", b"a", ws, ws + b"abc", b"\xff\xfe", b"ab\x00cd", b"\xe3\x81", "日本語テキスト".encode(),
        ws + b"a" * 300, ws + (b"ab" * 2000), b"zzzzqqqq", "▁▁▁".encode(),
        "é".encode() + b"\x80\x80" + "漢".encode()[:2],
        # NUL right after a piece with no children (base 0): must not step onto the root
        ws + b"x\x00y", b"x\x00y", b"q\x00\x00", ws + b"the\x00a\x00",
    ]


@pytest.mark.parametrize("name", ["test_model.model", "botchan_bpe1k.model"])
def test_edge_cases(name):
    mb = _read(os.path.join(GOLD, name))
    _compare(mb, _edge_sentences())
    _compare(mb, _edge_sentences(), force_general=True)


def test_unigram_known_answer_models():
    """Hand-built models in the style of unigram_model_test.cc:580-673:
    user-defined symbols, UNUSED pieces, ties."""
    pieces = base_pieces() + [
        ("a", 0.1, NORMAL), ("b", 0.2, NORMAL), ("c", 0.3, NORMAL), ("d", 0.4, NORMAL),
        ("ab", 0.5, NORMAL), ("cd", 0.6, NORMAL), ("abc", 0.7, UNUSED), ("bcd", 0.1, NORMAL),
        ("<tag>", 0.0, USER_DEFINED), ("▁", 0.0, NORMAL), ("▁a", -0.5, NORMAL),
        ("aa", 0.2, NORMAL), ("ba", 0.3, NORMAL),  # 0.1+0.2 vs 0.3: float ties
    ]
    mb = model(pieces, UNIGRAM)
    sents = [b"abcd", b"<tag>ab<tag>", b"abcabc", b"xyz", b"aaaa", b"abab",
             "▁ab▁cd".encode(), b"<ta", b"ba" * 50 + b"ab" * 50]
    _compare(mb, sents)
    _compare(mb, sents, force_general=True)


def test_bpe_known_answer_models():
    """bpe_model_test.cc style: ties on the leftmost pair, UNUSED resegment,
    user-defined symbols, chars outside the vocabulary."""
    pieces = base_pieces() + [
        ("ab", 0.0, NORMAL), ("cd", -0.1, NORMAL), ("abc", -0.2, NORMAL), ("a", -0.3, NORMAL),
        ("b", -0.4, NORMAL), ("c", -0.5, NORMAL), ("ABC", -0.5, NORMAL), ("abcdabcd", -0.5, NORMAL),
        ("q", -0.5, NORMAL), ("r", -0.5, NORMAL), ("qr", -0.5, UNUSED), ("d", -0.6, NORMAL),
        ("qrq", -0.7, NORMAL), ("aa", -0.05, NORMAL), ("bb", -0.05, NORMAL),
    ]
    mb = model(pieces, BPE)
    sents = [b"abcd", b"abcdabcd", b"aaaa", b"aabb", b"qrqr", b"xyzab", b"ABC", b"abcabcd" * 10]
    _compare(mb, sents)
    _compare(mb, sents, force_general=True)
    ud = model(pieces + [("<tag>", 0.0, USER_DEFINED)], BPE)
    _compare(ud, sents + [b"ab<tag>cd", b"<tag><tag>"])


@pytest.mark.parametrize("force_general", [False, True])
def test_reference_known_answers_on_gpu(force_general):
    """The reference's own unit-test expectations (tests/known_answers.py)."""
    import known_answers as KA
    for name, mb, exp in KA.cases():
        dm = S.DeviceModel(mb)
        dm.set_force_general(force_general)
        inputs = [KA.as_bytes(i) for i, _ in exp]
        buf, off = S.to_csr(inputs)
        ids, lens, to = dm.encode_csr_host(buf, off, with_lens=True)
        for k, (inp, want) in enumerate(exp):
            got = KA.split_pieces(inp, lens[int(to[k]):int(to[k + 1])])
            assert got == [KA.as_bytes(w) for w in want], (name, inp)


@pytest.mark.parametrize("model_name,text", [
    ("test_model.model", "botchan.txt"),
    ("test_model.model", "wagahaiwa_nekodearu.txt"),  # English 1k model on Japanese: long UNK runs
    ("test_ja_model.model", "wagahaiwa_nekodearu.txt"),
    ("botchan_bpe1k.model", "botchan.txt"),
    ("botchan_bpe1k.model", "wagahaiwa_nekodearu.txt"),
])
@pytest.mark.parametrize("opts", ["", "bos", "eos:reverse", "reverse:bos:eos", "bos:bos:eos:reverse:eos"])
def test_device_epilogue_vs_oracle(model_name, text, opts):
    """Raw lines → final ids entirely on the device (normalize + encode +
    spm_hip_finalize_ids: unk-run merge, bos/eos/reverse) == the oracle's
    SentencePieceProcessor::Encode(ids) with the same extra options."""
    mb = _read(os.path.join(GOLD, model_name))
    lines = O.read_lines_binary(os.path.join(GOLD, text))[:1500] + [b"", b" ", "▁".encode()]
    got = S.DeviceModel(mb).encode_lines_device(lines, opts)
    om = O.OracleModel(mb)
    om.set_extra_options(opts)
    want = om.encode_lines(lines)
    bad = [i for i in range(len(lines)) if got[i] != want[i]]
    assert not bad, "first mismatch at line %d: %r vs %r" % (bad[0], got[bad[0]], want[bad[0]])


def test_device_epilogue_errors():
    mb = _read(os.path.join(GOLD, "test_model.model"))
    dm = S.DeviceModel(mb)
    with pytest.raises(S.SpmError) as e:
        dm.encode_lines_device([b"abc"], "foo")
    assert e.value.code == 13
