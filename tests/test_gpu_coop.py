"""GPU parity of the wave-cooperative unigram kernel (csrc/coop_encode.hip):
one sentence per wavefront, the lattice walks of a sentence 64 at a time,
Viterbi over char starts with readlane broadcasts, backtrace through global
scratch.  With spm_hip_model_set_coop_min_nb(1) every sentence of a wide- or
char-kernel model takes it; results must equal the CPU oracle (the reference
Lattice / PopulateNodes / Viterbi restated, unigram_model.cc:147-261,
:535-604) bit for bit, ids and piece byte lengths.  Sentences it cannot take
(a leaf inside a UTF-8 char, more than 8 nodes at one position, malformed
UTF-8) must reach the general kernel and stay exact too."""
import os

import numpy as np
import pytest

import oracle_lib as O
import spm_amd as S
import synth
from model_builder import NORMAL, UNIGRAM, UNUSED, USER_DEFINED, base_pieces, model
import model_reader
from test_gpu_parity import _LONG_LAST, _compare, _edge_sentences, _read, _synth_model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")

pytestmark = pytest.mark.gpu


def _long_sentences(rng, n, lo, hi, alphabet):
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi))
        out.append(("▁" + "".join(alphabet[int(x)] for x in rng.integers(0, len(alphabet), L))).encode())
    return out


def _coop_compare(mb, sents, kernel):
    dm = S.DeviceModel(mb)
    assert dm.info().fast_variant == kernel
    dm.set_coop_min_nb(1)
    return _compare(mb, sents, dm=dm)


@pytest.mark.parametrize("extra,kernel", [(20, 2), (40, 2), (-9, 3), (-14, 3)])
def test_coop_every_sentence_vs_oracle(extra, kernel):
    """Every sentence through the cooperative kernel: synthetic ~25-char
    sentences, the edge cases (empty, NUL, 0xFF, broken UTF-8, 4 KB lines),
    long lines over several 64-byte windows, and a > 64-byte last sentence."""
    mb, extra_sents = _synth_model(extra)
    buf, off = synth.normalized(20000, seed=31)
    b = buf.tobytes()
    rng = np.random.default_rng(3)
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)] + _edge_sentences() + extra_sents
    sents += _long_sentences(rng, 300, 60, 3000, "abcdefghijklmnopqrstuvwxyz▁é")
    _coop_compare(mb, sents + [_LONG_LAST], kernel)


@pytest.mark.parametrize("extra", [20, -9])
def test_coop_near_tie_stress(extra):
    """Multi-char pieces one float ulp below their split: the Viterbi's
    first-lnode rule decides, which the cooperative kernel applies literally
    (no near-tie bookkeeping)."""
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
    pieces.append(("▁" + "q" * (extra - 3), -30.0, NORMAL) if extra > 0 else ("▁" + "é" * -extra, -30.0, NORMAL))
    mb = model(pieces, UNIGRAM)
    sents = _long_sentences(rng, 8000, 0, 40, alpha) + _long_sentences(rng, 200, 100, 2000, alpha)
    _coop_compare(mb, sents + [_LONG_LAST], 2 if extra > 0 else 3)


def test_coop_user_defined_unused_and_overflow():
    """USER_DEFINED scoring (length * max_score + 1.0), UNUSED pieces skipped
    (their position gets an UNK node), and a position with more than 8 prefix
    matches (general kernel)."""
    pieces = base_pieces() + [
        ("a", -1.0, NORMAL), ("b", -1.5, NORMAL), ("c", -2.0, NORMAL), ("ab", -1.2, NORMAL),
        ("abc", -0.5, USER_DEFINED), ("bc", -2.5, UNUSED), ("d", -3.0, UNUSED), ("é", -2.0, NORMAL),
        ("▁" + "q" * 25, -30.0, NORMAL),  # a 28-byte piece: char kernel
    ] + [("z" * k, -float(k), NORMAL) for k in range(1, 13)]  # 12 prefix matches of "zzz…"
    mb = model(pieces, UNIGRAM)
    rng = np.random.default_rng(9)
    sents = _long_sentences(rng, 3000, 0, 200, "abcdéz") + [b"z" * 40, b"abcabc" * 30, b"dddd", "é".encode() * 70]
    _coop_compare(mb, sents, 2)


def test_coop_four_byte_chars_windows_and_blocks():
    """Four-byte chars (a 192-byte window then holds 48 chars, so windows and
    the backtrace's 64-char blocks do not line up), pieces spanning them, and
    lines past 4096 chars (block starts past the first 64 come from the
    scratch, not the windows' register), through the dense node numbering."""
    pieces = base_pieces() + [
        ("a", -2.0, NORMAL), ("b", -2.5, NORMAL), ("😀", -3.0, NORMAL), ("🎉", -3.5, NORMAL),
        ("ab", -2.2, NORMAL), ("a😀", -4.0, NORMAL), ("😀😀", -5.0, NORMAL), ("😀b🎉", -6.0, NORMAL),
        ("🎉a", -4.5, NORMAL), ("ba😀", -5.5, NORMAL), ("é", -3.0, NORMAL), ("é😀", -4.2, NORMAL),
        ("▁" + "q" * 25, -30.0, NORMAL),  # a 28-byte piece: char kernel, which hands lines over
    ]
    mb = model(pieces, UNIGRAM)
    rng = np.random.default_rng(21)
    alpha = ["a", "b", "😀", "🎉", "é", "x"]
    sents = []
    for lo, hi, n in ((0, 40, 2000), (40, 400, 300), (400, 3000, 60), (4100, 6000, 6)):
        for _ in range(n):
            L = int(rng.integers(lo, hi))
            sents.append(("▁" + "".join(alpha[int(x)] for x in rng.integers(0, len(alpha), L))).encode())
    sents += [("😀" * k).encode() for k in (47, 48, 49, 63, 64, 65, 127, 128, 129, 4200)]
    st = _coop_compare(mb, sents, 2)
    assert st.general_path >= len(sents) // 2


def test_coop_ja_golden_all_sentences():
    """The reference's Japanese model on its own corpus (paragraphs up to
    33 KB), every line through the cooperative kernel, vs the golden ids."""
    mb = open(os.path.join(GOLD, "test_ja_model.model"), "rb").read()
    lines = O.read_lines_binary(os.path.join(GOLD, "wagahaiwa_nekodearu.txt"))
    norm = O.OracleModel(mb).normalize(lines)
    st = _coop_compare(mb, norm, 3)
    assert st.general_path >= len([s for s in norm if len(s) > 0]) // 2


@pytest.mark.parametrize("slab_chars", [0, 300])
def test_coop_wave_slabs_vs_oracle(slab_chars):
    """Per-wave scratch slabs (the layout a large batch gets): every line of
    the Japanese corpus plus long ASCII / mixed lines; with 300-char slabs the
    lines of more chars must leave the cooperative kernel for the general
    kernel and stay exact, and with the default slabs (16384 chars) the 33 KB
    paragraph (11184 chars) stays in it."""
    mb = open(os.path.join(GOLD, "test_ja_model.model"), "rb").read()
    lines = O.read_lines_binary(os.path.join(GOLD, "wagahaiwa_nekodearu.txt"))
    norm = O.OracleModel(mb).normalize(lines)
    rng = np.random.default_rng(12)
    norm += _long_sentences(rng, 40, 250, 900, "abcdefgh▁é")
    dm = S.DeviceModel(mb)
    dm.set_coop_min_nb(1)
    dm.set_coop_slab(1, slab_chars)
    st = _compare(mb, norm, dm=dm)
    assert st.general_path >= len([s for s in norm if len(s) > 0]) // 2
    long_lines = sum(1 for s in norm if len(s.decode("utf-8", "replace")) > 300)
    if slab_chars:
        assert st.coop_rest >= long_lines > 0, (st.coop_rest, long_lines)
    else:
        assert st.coop_rest < long_lines, (st.coop_rest, long_lines)
    dm.set_coop_slab(2)
    _compare(mb, norm[:600], dm=dm)


@pytest.mark.parametrize("model_path", [os.path.join(ROOT, "data", "synth32k_unigram.model"),
                                        os.path.join(GOLD, "test_ja_model.model"),
                                        os.path.join(GOLD, "test_model.model")])
def test_coop_small_host_calls(model_path):
    """spm_hip_encode_batch_host with 1..16 sentences takes the one-block
    cooperative kernel (pinned input, outputs and completion word in host
    memory): bit-exact vs the oracle on single lines, short batches, empty
    and broken lines (re-run on the lane kernels) and multi-window lines."""
    mb = open(model_path, "rb").read()
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    if "ja" in model_path:
        lines = O.read_lines_binary(os.path.join(GOLD, "wagahaiwa_nekodearu.txt"))
        pool = om.normalize(lines)
    else:
        buf, off = synth.normalized(2000, seed=77)
        b = buf.tobytes()
        pool = [b[int(off[i]):int(off[i + 1])] for i in range(2000)]
        pool += _long_sentences(np.random.default_rng(1), 50, 100, 3000, "abcdefghij▁")
    pool += [b"", b"\xff", b"\xe3\x81", "▁é".encode() * 40]
    rng = np.random.default_rng(2)
    for t in range(400):
        n = 1 if t % 3 else int(rng.integers(1, 17))
        batch = [pool[int(x)] for x in rng.integers(0, len(pool), n)]
        if t < 4:
            batch = [pool[-1 - t]]
        buf, off = S.to_csr(batch)
        ids, lens, tok = dm.encode_csr_host(buf, off, with_lens=True)
        rids, rlens, rtok = om.encode_normalized_csr(buf, off, with_lens=True)
        assert np.array_equal(tok, rtok) and np.array_equal(ids, rids) and np.array_equal(lens, rlens), (t, n)
    dm.close()


@pytest.mark.parametrize("model_path,corpus", [
    (os.path.join(ROOT, "data", "synth32k_unigram.model"), None),
    (os.path.join(GOLD, "test_model.model"), "botchan.txt"),
    (os.path.join(GOLD, "test_ja_model.model"), "wagahaiwa_nekodearu.txt")])
def test_raw_small_lines_vs_oracle(model_path, corpus):
    """spm_hip_encode_raw_small_host (coop_raw_kernel: the device normalizer's
    state machine fed by wave-parallel NormalizePrefix, the cooperative
    encode, the unknown-run merge) vs the oracle's Encode(line, &ids) on raw
    lines: 1..16-line calls, edge lines (empty, spaces only, tabs and runs of
    spaces, malformed UTF-8, NUL, unknown chars, > 1024 bytes -> not taken)."""
    mb = open(model_path, "rb").read()
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    if corpus:
        pool = [l for l in O.read_lines_binary(os.path.join(GOLD, corpus)) if len(l) <= 1024]
    else:
        rng = np.random.default_rng(4)
        words = ["hello", "world", "the", "of", "tokenizer", "GPU", "x", "éà", "ü", "naïve"]
        pool = [" ".join(words[int(k)] for k in rng.integers(0, len(words), int(rng.integers(1, 30))))
                .encode() for _ in range(500)]
    pool += [b"", b"   ", b"\t a  b \t", b"  lead", b"trail   ", b"\xff\xfe", b"a\x00b", b"\xe3\x81",
             "☃ ♞ 𝄞 ∀".encode(), b"x" * 1000, "▁▁ ▁".encode()]
    rng = np.random.default_rng(8)
    taken = 0
    for t in range(300):
        n = 1 if t % 2 else int(rng.integers(1, 17))
        batch = [pool[int(x)] for x in rng.integers(0, len(pool), n)]
        if t < 11:
            batch = [pool[-1 - t]]
        got = dm.encode_raw_small(batch)
        want = om.encode_lines(batch)
        if got is None:
            continue
        taken += 1
        assert [list(map(int, g)) for g in got] == [list(map(int, w)) for w in want], (t, batch)
    assert taken >= 250, taken
    assert dm.encode_raw_small([b"y" * 1500]) is None  # past the prefix table: not taken
    dm.close()


def _ws_fuzz_lines(seed, n):
    """Whitespace-heavy raw lines: runs of spaces and tabs, leading and
    trailing runs, literal U+2581, ideographic spaces and NFKC-folded chars
    (U+00A8 -> space + combining diaeresis, a ligature, fullwidth letters),
    lines long enough to cross the normalizer's 64-position blocks."""
    rng = np.random.default_rng(seed)
    toks = [" ", "  ", "   ", "\t", "a", "bc", "hello", "é", "▁", "▁▁", "　", "¨", "ﬁ", "ＡＢ", "x" * 70,
            "the", "q", "é" * 5]
    out = [b"", b" ", b"  \t ", "▁".encode(), " ▁ ".encode(), "　a　".encode(), "¨".encode(),
           " ¨ ".encode(), ("a" + " " * 130 + "b").encode(), (" " * 64 + "x").encode(), ("x" + " " * 64).encode()]
    for _ in range(n):
        s = "".join(toks[int(k)] for k in rng.integers(0, len(toks), int(rng.integers(1, 40))))
        out.append(s.encode()[:1000])
    return out


@pytest.mark.parametrize("flags", [
    dict(),
    dict(remove_extra_whitespaces=False),
    dict(add_dummy_prefix=False),
    dict(treat_ws_as_suffix=True),
    dict(escape_whitespaces=False),
    dict(remove_extra_whitespaces=False, add_dummy_prefix=False, treat_ws_as_suffix=True)])
def test_raw_small_normalizer_flags_vs_oracle(flags):
    """coop_raw_kernel's wave-parallel normalizer (chain walk, leading /
    repeated / trailing whitespace, dummy prefix as prefix or suffix,
    escaping) vs the oracle's Normalizer::Normalize + Encode on every flag
    combination the spec has (normalizer.cc:88-211), identity charsmap."""
    pcs = [(p, s, t) for p, s, t in model_reader.read_pieces(_read(os.path.join(ROOT, "data", "synth32k_unigram.model")))]
    mb = model(pcs, UNIGRAM, **flags)
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    lines = _ws_fuzz_lines(11, 400)
    taken = 0
    for i in range(0, len(lines), 4):
        batch = lines[i:i + 4] if (i // 4) % 2 else lines[i:i + 1]
        got = dm.encode_raw_small(batch)
        if got is None:
            continue
        taken += 1
        want = om.encode_lines(batch)
        assert [list(map(int, g)) for g in got] == [list(map(int, w)) for w in want], (flags, batch)
    assert taken >= 90, taken
    dm.close()


@pytest.mark.parametrize("model_name", ["test_model.model", "test_ja_model.model"])
def test_raw_small_charsmap_ws_fuzz_vs_oracle(model_name):
    """The same whitespace fuzz through a real charsmap (nmt_nfkc): folded
    spaces and multi-byte replacements meet the whitespace rules."""
    mb = open(os.path.join(GOLD, model_name), "rb").read()
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    lines = _ws_fuzz_lines(12, 300)
    taken = 0
    for x in lines:
        got = dm.encode_raw_small([x])
        if got is None:
            continue
        taken += 1
        want = om.encode_lines([x])
        assert [list(map(int, g)) for g in got] == [list(map(int, w)) for w in want], x
    assert taken >= 250, taken
    dm.close()


def test_small_calls_resident_server_idle_and_kind_switch():
    """The resident small-call server (coop_service_kernel): calls back to
    back, calls after it has idled out (SPM_HIP_SERVICE_IDLE_US, 2 ms: the
    next call relaunches it), raw-line and normalized calls interleaved (two
    call kinds, one server), and a batch whose buffers grow (the server is
    restarted with the new tables) -- every result equal to the oracle's."""
    import time
    mb = open(os.path.join(GOLD, "test_model.model"), "rb").read()
    dm = S.DeviceModel(mb)
    om = O.OracleModel(mb)
    lines = O.read_lines_binary(os.path.join(GOLD, "botchan.txt"))[:300]
    norm = om.normalize(lines)
    rng = np.random.default_rng(31)
    for t in range(240):
        if t % 40 == 39:
            time.sleep(0.01)  # past the idle timeout
        k = int(rng.integers(0, len(lines)))
        if t % 3 == 0:
            got = dm.encode_raw_small([lines[k]])
            assert got is not None and [list(map(int, g)) for g in got] == \
                [list(map(int, w)) for w in om.encode_lines([lines[k]])], t
        else:
            m = 1 if t % 3 == 1 else int(rng.integers(2, 17))
            batch = [norm[(k + j) % len(norm)] for j in range(m)]
            if t == 200:
                batch = [b"\xe2\x96\x81" + b"x" * 3000]  # grows the small-call buffers
            buf, off = S.to_csr(batch)
            ids, lens, tok = dm.encode_csr_host(buf, off, with_lens=True)
            rids, rlens, rtok = om.encode_normalized_csr(buf, off, with_lens=True)
            assert np.array_equal(tok, rtok) and np.array_equal(ids, rids) and np.array_equal(lens, rlens), t
    dm.close()
