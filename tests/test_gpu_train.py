"""GPU: the unigram trainer path (spm_train) against the oracle.

* spm_hip_seed_mine (MakeSeedSentencePieces on the device) — seed pieces and
  their float scores bit-identical to the oracle's literal esaxx restatement,
  over several corpora and IsValidSentencePiece flag settings;
* lib/spm_train end to end — the .model piece table (piece, score bits, type)
  and the .vocab text identical to the oracle trainer's, and the reference's
  own EndToEnd known answer (unigram_model_trainer_test.cc:47-86).
"""
import collections
import json
import os
import subprocess

import numpy as np
import pytest

import model_reader
import oracle_lib as O
import synth
from test_trainer_cpu import (BPE_BASIC, BPE_KAT_ARGS, BPE_KAT_WANT, KAT_ARGS, KAT_TEXT, KAT_WANT,
                              bpe_basic_args)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
LIB = os.path.join(ROOT, "sentencepiece-comments_amd", "lib")
TRAIN = os.path.join(LIB, "spm_train")
ENCODE = os.path.join(LIB, "spm_encode")
RULES = os.path.join(ROOT, "data", "normalization")
pytestmark = pytest.mark.gpu


def _lines(name):
    return O.read_lines_binary(os.path.join(GOLD, name))


def _charsmap(rule):
    return b"" if rule == "identity" else open(os.path.join(RULES, rule + ".bin"), "rb").read()


def _synth_file(tmp_path, n, seed=7):
    sents = synth.lines(n, seed=seed)
    p = tmp_path / ("synth_%d.txt" % n)
    p.write_bytes(b"".join(s + b"\n" for s in sents))
    return str(p)


def _rule_of(args):
    for a in args.split():
        if a.startswith("--normalization_rule_name="):
            return a.split("=", 1)[1]
    return "nmt_nfkc"


def _flag(args, key, default):
    for a in args.split():
        if a.startswith("--" + key + "="):
            return a.split("=", 1)[1]
    return default


SEED_CASES = [
    ("wagahaiwa_nekodearu.txt", KAT_ARGS),
    ("botchan.txt", "--vocab_size=1000 --normalization_rule_name=nfkc"),
    ("botchan.txt", "--vocab_size=1000 --normalization_rule_name=identity --split_by_whitespace=false"),
    ("botchan.txt", "--vocab_size=1000 --normalization_rule_name=nfkc --split_by_number=false "
                    "--treat_whitespace_as_suffix=true"),
    ("botchan.txt", "--vocab_size=1000 --normalization_rule_name=nfkc --max_sentencepiece_length=4 "
                    "--seed_sentencepiece_size=3000"),
    ("wagahaiwa_nekodearu.txt", "--vocab_size=8000 --normalization_rule_name=nfkc "
                                "--split_by_unicode_script=false"),
]


@pytest.mark.parametrize("corpus,args", SEED_CASES)
def test_seed_mine_matches_oracle(corpus, args):
    import spm_amd
    ot = O.OracleTrainer(args, _lines(corpus), _charsmap(_rule_of(args)))
    sents, freq = ot.sentences()
    want_p, want_s = ot.seeds()
    cnt = collections.Counter()
    for s, f in zip(sents, freq):
        for ch in s.decode():
            if ch != "▅":
                cnt[ord(ch)] += int(f)
    chars = sorted(cnt)
    got_p, got_s, st = spm_amd.seed_mine(
        sents, chars, [cnt[c] for c in chars],
        max_sentencepiece_length=int(_flag(args, "max_sentencepiece_length", 16)),
        split_by_unicode_script=_flag(args, "split_by_unicode_script", "true") == "true",
        split_by_number=_flag(args, "split_by_number", "true") == "true",
        split_by_whitespace=_flag(args, "split_by_whitespace", "true") == "true",
        treat_whitespace_as_suffix=_flag(args, "treat_whitespace_as_suffix", "false") == "true",
        seed_sentencepiece_size=int(_flag(args, "seed_sentencepiece_size", 1000000)))
    assert len(got_p) == len(want_p)
    bad = [i for i in range(len(want_p)) if got_p[i] != want_p[i]]
    assert not bad, [(i, got_p[i].decode(), want_p[i].decode()) for i in bad[:5]]
    assert np.array_equal(got_s.view(np.uint32), want_s.view(np.uint32))
    assert st["num_chars"] == len(chars)


def test_seed_mine_synthetic_large():
    """100k synthetic sentences (c2/c5 distribution), identity rule."""
    import spm_amd
    lines = synth.lines(100_000, seed=11)
    args = "--vocab_size=8000 --normalization_rule_name=identity"
    ot = O.OracleTrainer(args, lines)
    sents, freq = ot.sentences()
    want_p, want_s = ot.seeds()
    cnt = collections.Counter()
    for s in sents:
        cnt.update(ord(c) for c in s.decode())
    chars = sorted(cnt)
    got_p, got_s, st = spm_amd.seed_mine(sents, chars, [cnt[c] for c in chars])
    assert got_p == want_p
    assert np.array_equal(got_s.view(np.uint32), want_s.view(np.uint32))
    assert st["candidates"] >= len(want_p) - len(chars)


def _long_repeat_lines():
    """botchan plus long shared cores (34-38 and 270-290 chars) that recur
    with different right contexts, so the suffix tree has branching nodes of
    that depth (> 32: the E-step's long-piece path; > 255: the uint16 LCP path
    of the seed miner)."""
    base = _lines("botchan.txt")[:1200]
    rng = np.random.default_rng(9)
    out = list(base)
    k = 0
    for n in (34, 36, 38, 270, 280, 290):
        core = bytes(rng.choice(list(b"abcdefghij"), size=n).tolist())
        for tail in (b"Q", b"RS", b"T", b"UV"):
            out.insert(37 * k + 5, core + tail)
            k += 1
    return out


@pytest.mark.parametrize("max_len", [40, 300])
def test_seed_mine_long_max_sentencepiece_length(max_len):
    """max_sentencepiece_length beyond 32 / 254 (TrainerSpec allows 1..512,
    trainer_interface.cc:74)."""
    import spm_amd
    args = ("--vocab_size=1000 --normalization_rule_name=identity --split_by_whitespace=false "
            "--max_sentencepiece_length=%d" % max_len)
    ot = O.OracleTrainer(args, _long_repeat_lines())
    sents, freq = ot.sentences()
    want_p, want_s = ot.seeds()
    assert max(len(p.decode()) for p in want_p) >= (270 if max_len == 300 else 34)
    cnt = collections.Counter()
    for s, f in zip(sents, freq):
        for ch in s.decode():
            if ch != "▅":
                cnt[ord(ch)] += int(f)
    chars = sorted(cnt)
    got_p, got_s, st = spm_amd.seed_mine(sents, chars, [cnt[c] for c in chars], max_sentencepiece_length=max_len,
                                         split_by_whitespace=False)
    assert got_p == want_p
    assert np.array_equal(got_s.view(np.uint32), want_s.view(np.uint32))


def _train_gpu(tmp_path, input_path, args, tag, env=None):
    prefix = str(tmp_path / tag)
    cmd = [TRAIN, "--input=" + input_path, "--model_prefix=" + prefix] + args.split()
    p = subprocess.run(cmd, capture_output=True, timeout=600, env=None if env is None else {**os.environ, **env})
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-3000:]
    # pruning NBest(2) ran on the device (spm_hip_prune_nbest) for every piece
    assert b"outgrew the device slab" not in p.stderr
    em = [l for l in p.stderr.decode().splitlines() if l.startswith("EM sub_iter=")]
    _train_gpu.last_log = p.stderr.decode(errors="replace")
    _train_gpu.last_stdout = p.stdout.decode(errors="replace")
    return prefix, em


def _vocab_text(pieces, scores):
    return b"".join(p + b"\t" + ("%g" % float(s)).encode() + b"\n" for p, s in zip(pieces, scores))


TRAIN_CASES = [
    ("wagahaiwa_nekodearu.txt", KAT_ARGS),
    ("botchan.txt", "--vocab_size=1000 --normalization_rule_name=nfkc --num_threads=1"),
    ("botchan.txt", "--vocab_size=2000 --normalization_rule_name=nfkc --num_threads=8 "
                    "--split_by_whitespace=false"),
]


@pytest.mark.parametrize("corpus,args", TRAIN_CASES)
def test_spm_train_matches_oracle(corpus, args, tmp_path):
    path = os.path.join(GOLD, corpus)
    prefix, em = _train_gpu(tmp_path, path, args, "m")
    ot = O.OracleTrainer(args, _lines(corpus), _charsmap(_rule_of(args)))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))
    assert [g[2] for g in got] == list(wt)
    assert open(prefix + ".vocab", "rb").read() == _vocab_text(wp, ws)
    want_em = ot.em_log()
    assert [l.split(" num_tokens/piece")[0] for l in em] == want_em


def test_spm_train_known_answer(tmp_path):
    """unigram_model_trainer_test.cc:47-86 through spm_train + spm_encode."""
    prefix, _ = _train_gpu(tmp_path, os.path.join(GOLD, "wagahaiwa_nekodearu.txt"), KAT_ARGS, "kat")
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert len(got) == 8000
    src = tmp_path / "kat.txt"
    src.write_bytes(KAT_TEXT.encode() + b"\n")
    out = subprocess.run([ENCODE, "--model=" + prefix + ".model", "--output_format=piece", str(src)],
                         capture_output=True, timeout=120)
    assert out.returncode == 0
    assert out.stdout.decode().rstrip("\n") == KAT_WANT


def test_spm_train_synthetic(tmp_path):
    """c5-shaped corpus (synthetic, identity rule): 30k lines, vocab 2000."""
    path = _synth_file(tmp_path, 30_000)
    args = "--vocab_size=2000 --normalization_rule_name=identity --num_threads=16"
    prefix, em = _train_gpu(tmp_path, path, args, "syn")
    ot = O.OracleTrainer(args, O.read_lines_binary(path))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))


@pytest.mark.parametrize("stop_before", [0, 2])
def test_spm_train_em_checkpoint_resume(stop_before, tmp_path):
    """--em_checkpoint / --resume_from (trainer.cc WriteEmCheckpoint): a run
    stopped before EM round r and resumed from its checkpoint gives the
    uninterrupted run's piece table and .vocab, and the same EM log from
    round r on (round 0's checkpoint is the seed list: the resumed run mines
    no seeds)."""
    path = os.path.join(GOLD, "botchan.txt")
    args = "--vocab_size=1000 --normalization_rule_name=nfkc --num_threads=8"
    full, em_full = _train_gpu(tmp_path, path, args, "full")
    ck = str(tmp_path / "em.ck")
    p = subprocess.run([TRAIN, "--input=" + path, "--model_prefix=" + str(tmp_path / "cut"), "--em_checkpoint=" + ck]
                       + args.split(), capture_output=True, timeout=600,
                       env={**os.environ, "SPM_HIP_EM_STOP_BEFORE": str(stop_before)})
    assert p.returncode != 0 and b"stopped before EM round %d" % stop_before in p.stderr
    assert not os.path.exists(str(tmp_path / "cut.model"))
    head = open(ck, "rb").read(28)
    assert head[:8] == b"SPMEMCK1" and int.from_bytes(head[8:12], "little") == stop_before
    res, em_res = _train_gpu(tmp_path, path, args + " --resume_from=" + ck, "res")
    assert "Resumed EM round %d" % stop_before in _train_gpu.last_log
    if stop_before == 0:
        assert "Initialized" not in _train_gpu.last_log  # no seed mining
    got = model_reader.read_pieces(open(res + ".model", "rb").read())
    want = model_reader.read_pieces(open(full + ".model", "rb").read())
    assert [g[0] for g in got] == [w[0] for w in want]
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          np.array([w[1] for w in want], dtype=np.float32).view(np.uint32))
    assert open(res + ".vocab", "rb").read() == open(full + ".vocab", "rb").read()
    assert em_res == em_full[2 * stop_before:]  # num_sub_iterations = 2


def test_spm_train_resume_rejects_another_corpus(tmp_path):
    path = os.path.join(GOLD, "botchan.txt")
    args = "--vocab_size=1000 --normalization_rule_name=nfkc --num_threads=8"
    ck = str(tmp_path / "em.ck")
    subprocess.run([TRAIN, "--input=" + path, "--model_prefix=" + str(tmp_path / "cut"), "--em_checkpoint=" + ck]
                   + args.split(), capture_output=True, timeout=600, env={**os.environ, "SPM_HIP_EM_STOP_BEFORE": "1"})
    other = _synth_file(tmp_path, 2000)
    p = subprocess.run([TRAIN, "--input=" + other, "--model_prefix=" + str(tmp_path / "o"), "--resume_from=" + ck]
                       + args.split(), capture_output=True, timeout=600)
    assert p.returncode != 0 and b"is of another corpus" in p.stderr


def test_spm_train_timings_peak_device_bytes(tmp_path):
    """--timings reports the run's device high-water mark and each stage's
    (csrc/scratch_cache.cc DevMalloc accounting): every stage holds at least
    the corpus and the run's peak is the largest stage peak."""
    path = _synth_file(tmp_path, 30_000)
    size = os.path.getsize(path)
    cmd = [TRAIN, "--input=" + path, "--model_prefix=" + str(tmp_path / "pk"), "--vocab_size=2000",
           "--normalization_rule_name=identity", "--num_threads=16", "--timings"]
    p = subprocess.run(cmd, capture_output=True, timeout=600)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-3000:]
    tm = json.loads(p.stdout.decode().strip().splitlines()[-1])
    st = tm["stage_peak_bytes"]
    assert len(st) == 4 and tm["peak_device_bytes"] == max(st)
    assert min(st) > 0 and st[1] >= size // 2


def test_spm_train_synthetic_vocab_32k(tmp_path):
    """c5 at its stated vocab: 200k synthetic lines, --vocab_size=32000,
    identity rule, 16 E-step buckets; .model piece/score bits, types and
    .vocab bytes identical to the oracle trainer's."""
    path = _synth_file(tmp_path, 200_000, seed=1234)
    args = "--model_type=unigram --vocab_size=32000 --normalization_rule_name=identity --num_threads=16"
    prefix, em = _train_gpu(tmp_path, path, args, "syn32k")
    ot = O.OracleTrainer(args, O.read_lines_binary(path))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert len(got) == 32000
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))
    assert [g[2] for g in got] == list(wt)
    assert open(prefix + ".vocab", "rb").read() == _vocab_text(wp, ws)
    assert [l.split(" num_tokens/piece")[0] for l in em] == ot.em_log()


def test_spm_train_long_pieces(tmp_path):
    """--max_sentencepiece_length=40 with no whitespace split: seeds and EM
    pieces of 32+ chars run the E-step's general path (node-count pre-pass) in
    PARITY mode; the model equals the oracle trainer's."""
    lines = _long_repeat_lines()
    path = tmp_path / "long.txt"
    path.write_bytes(b"\n".join(lines) + b"\n")
    args = ("--vocab_size=1500 --normalization_rule_name=identity --split_by_whitespace=false "
            "--max_sentencepiece_length=40 --num_threads=8")
    prefix, em = _train_gpu(tmp_path, str(path), args, "long")
    ot = O.OracleTrainer(args, O.read_lines_binary(str(path)))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))
    assert [l.split(" num_tokens/piece")[0] for l in em] == ot.em_log()


MULTI_CASES = [
    ("botchan.txt", "--vocab_size=1000 --normalization_rule_name=nfkc --num_threads=16", 2),
    ("botchan.txt", "--vocab_size=1000 --normalization_rule_name=nfkc --num_threads=8", 3),
    ("botchan.txt", "--vocab_size=2000 --normalization_rule_name=nfkc --num_threads=8 "
                    "--split_by_whitespace=false", 4),
    ("wagahaiwa_nekodearu.txt", KAT_ARGS, 8),
]


@pytest.mark.parametrize("corpus,args,ranks", MULTI_CASES)
def test_spm_train_num_gpus_matches_oracle(corpus, args, ranks, tmp_path):
    """spm_train --num_gpus=N: every E-step and pruning Viterbi sharded over N
    ranks by bucket ownership (csrc/shard_plan.h), reduced onto rank 0.  On a
    1-GPU box the ranks share the device and reduce through the host; on a
    node with >= N GPUs the same code reduces over RCCL.  The .model, .vocab
    and EM log equal the oracle trainer's at the same num_threads (the
    reference's output), i.e. rank count never changes a bit."""
    path = os.path.join(GOLD, corpus)
    prefix, em = _train_gpu(tmp_path, path, args + " --num_gpus=%d" % ranks, "r%d" % ranks)
    ot = O.OracleTrainer(args, _lines(corpus), _charsmap(_rule_of(args)))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))
    assert [g[2] for g in got] == list(wt)
    assert open(prefix + ".vocab", "rb").read() == _vocab_text(wp, ws)
    assert [l.split(" num_tokens/piece")[0] for l in em] == ot.em_log()


def _device_count():
    import torch
    return torch.cuda.device_count()  # (does not initialise the GPU on this image)


@pytest.mark.skipif(_device_count() < 2, reason="the RCCL reduction needs >= 2 GPUs (pool boxes have one)")
@pytest.mark.parametrize("mode", ["parity", "fast"])
def test_spm_train_num_gpus_rccl(mode, tmp_path):
    """--num_gpus=2 on a node with >= 2 GPUs: one rank per device, the
    accumulators meet on rank 0 over RCCL (PARITY: owned bucket rows by
    ncclSend/Recv; FAST: ncclReduce).  PARITY must equal the oracle exactly;
    FAST must equal the 1-GPU FAST run's pieces."""
    path = os.path.join(GOLD, "botchan.txt")
    args = "--vocab_size=1000 --normalization_rule_name=nfkc --num_threads=16"
    if mode == "fast":
        p1, _ = _train_gpu(tmp_path, path, args + " --estep_mode=fast", "f1")
        p2, _ = _train_gpu(tmp_path, path, args + " --estep_mode=fast --num_gpus=2", "f2")
        assert "reduction RCCL" in _train_gpu.last_log
        a = [g[0] for g in model_reader.read_pieces(open(p1 + ".model", "rb").read())]
        b = [g[0] for g in model_reader.read_pieces(open(p2 + ".model", "rb").read())]
        assert len(set(a) & set(b)) >= 990
        return
    prefix, em = _train_gpu(tmp_path, path, args + " --num_gpus=2", "r2")
    assert "reduction RCCL" in _train_gpu.last_log
    ot = O.OracleTrainer(args, _lines("botchan.txt"), _charsmap(_rule_of(args)))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))
    assert [l.split(" num_tokens/piece")[0] for l in em] == ot.em_log()


def test_spm_train_num_gpus_fast_mode(tmp_path):
    """FAST E-step (fp64 sums) over 2 ranks trains a full vocabulary; the
    pieces overlap the PARITY model's almost entirely."""
    path = os.path.join(GOLD, "botchan.txt")
    base = "--vocab_size=1000 --normalization_rule_name=nfkc --num_threads=16"
    p1, _ = _train_gpu(tmp_path, path, base, "par")
    p2, _ = _train_gpu(tmp_path, path, base + " --estep_mode=fast --num_gpus=2", "fast2")
    a = {g[0] for g in model_reader.read_pieces(open(p1 + ".model", "rb").read())}
    b = {g[0] for g in model_reader.read_pieces(open(p2 + ".model", "rb").read())}
    assert len(b) == 1000 and len(a & b) >= 950


def test_spm_train_errors(tmp_path):
    p = subprocess.run([TRAIN, "--input=/nonexistent.txt", "--model_prefix=" + str(tmp_path / "x")],
                       capture_output=True, timeout=120)
    assert p.returncode != 0
    p = subprocess.run([TRAIN, "--input=" + os.path.join(GOLD, "botchan.txt"),
                        "--model_prefix=" + str(tmp_path / "x"), "--model_type=word"],
                       capture_output=True, timeout=120)
    assert p.returncode != 0
    p = subprocess.run([TRAIN, "--input=" + os.path.join(GOLD, "botchan.txt"),
                        "--model_prefix=" + str(tmp_path / "x"), "--vocab_size=10"],
                       capture_output=True, timeout=120)
    assert p.returncode != 0


def _crafted_lines():
    """botchan plus the LoadSentences edge cases: whitespace-only lines (empty
    after normalization → swap-with-last removal), meta pieces in the text
    (GlobalReplace → tab → UNK char), NUL bytes, tabs, U+2585 lines (skipped),
    over-long lines, rare chars."""
    base = O.read_lines_binary(os.path.join(GOLD, "botchan.txt"))[:1500]
    extra = [b"   ", b"\t", "<s> hello </s> world".encode(), b"a <user> b<user>c", b"nul\x00byte here",
             "rare ▅ skipped".encode(), b"x" * 3000, "ｱｲｳ Ⅷ ① ﬁ".encode(), b"\xff\xfe broken",
             "ǅ Ǆ ǆ ἀ ἁ ἂ".encode(), b"  ", b"tab\tinside"]
    out = []
    for i, l in enumerate(base):
        out.append(l)
        if i % 97 == 0:
            out.append(extra[(i // 97) % len(extra)])
    return out


@pytest.mark.parametrize("args", [
    "--vocab_size=800 --normalization_rule_name=nfkc --character_coverage=0.98 "
    "--user_defined_symbols=<user> --control_symbols=<ctrl> --max_sentence_length=2048 --num_threads=4",
    "--vocab_size=800 --normalization_rule_name=identity --split_by_whitespace=false --num_threads=3",
    "--vocab_size=600 --normalization_rule_name=nfkc --input_sentence_size=700 --num_threads=2",
    "--vocab_size=600 --normalization_rule_name=nfkc --input_sentence_size=700 "
    "--shuffle_input_sentence=false --num_threads=2",
])
def test_spm_train_load_edge_cases(args, tmp_path):
    lines = _crafted_lines()
    path = tmp_path / "crafted.txt"
    path.write_bytes(b"\n".join(lines) + b"\n")
    prefix, em = _train_gpu(tmp_path, str(path), args, "edge")
    ot = O.OracleTrainer(args, O.read_lines_binary(str(path)), _charsmap(_rule_of(args)))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))
    assert [l.split(" num_tokens/piece")[0] for l in em] == ot.em_log()


def test_spm_train_tsv(tmp_path):
    words = collections.Counter()
    for l in O.read_lines_binary(os.path.join(GOLD, "botchan.txt")):
        words.update(l.split())
    path = tmp_path / "words.tsv"
    path.write_bytes(b"".join(w + b"\t" + str(c).encode() + b"\n" for w, c in sorted(words.items())))
    args = "--vocab_size=1000 --normalization_rule_name=nfkc --input_format=tsv --num_threads=8"
    prefix, em = _train_gpu(tmp_path, str(path), args, "tsv")
    ot = O.OracleTrainer(args, O.read_lines_binary(str(path)), _charsmap("nfkc"))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))


# ---- BPE trainer (bpe_model_trainer.cc; device pair census + host merges) ----

def _check_vs_oracle(prefix, args, lines):
    ot = O.OracleTrainer(args, lines, _charsmap(_rule_of(args)))
    wp, ws, wt = ot.train()
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert [g[0] for g in got] == wp
    assert np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                          ws.view(np.uint32))
    assert [g[2] for g in got] == list(wt)
    assert open(prefix + ".vocab", "rb").read() == _vocab_text(wp, ws)


@pytest.mark.parametrize("lines,size,uds,want", BPE_BASIC)
def test_spm_train_bpe_basic_known_answer(lines, size, uds, want, tmp_path):
    """bpe_model_trainer_test.cc BasicTest through spm_train --model_type=bpe."""
    src = tmp_path / "in.txt"
    src.write_bytes(b"".join(l.encode() + b"\n" for l in lines))
    prefix, _ = _train_gpu(tmp_path, str(src), bpe_basic_args(size, uds), "b")
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert " ".join(g[0].decode() for g in got[3:]) == want


def test_spm_train_bpe_known_answer(tmp_path):
    """bpe_model_trainer_test.cc EndToEndTest through spm_train + spm_encode."""
    prefix, _ = _train_gpu(tmp_path, os.path.join(GOLD, "wagahaiwa_nekodearu.txt"), BPE_KAT_ARGS, "bkat")
    got = model_reader.read_pieces(open(prefix + ".model", "rb").read())
    assert len(got) == 8000
    src = tmp_path / "kat.txt"
    src.write_bytes(KAT_TEXT.encode() + b"\n")
    out = subprocess.run([ENCODE, "--model=" + prefix + ".model", "--output_format=piece", str(src)],
                         capture_output=True, timeout=120)
    assert out.returncode == 0
    assert out.stdout.decode().rstrip("\n") == BPE_KAT_WANT
    _check_vs_oracle(prefix, BPE_KAT_ARGS, _lines("wagahaiwa_nekodearu.txt"))


@pytest.mark.parametrize("corpus,args", [
    ("botchan.txt", "--model_type=bpe --vocab_size=1000 --normalization_rule_name=nfkc"),
    ("botchan.txt", "--model_type=bpe --vocab_size=2000 --normalization_rule_name=nfkc "
                    "--split_by_whitespace=false"),
    ("botchan.txt", "--model_type=bpe --vocab_size=1500 --normalization_rule_name=nfkc "
                    "--treat_whitespace_as_suffix=true --max_sentencepiece_length=8"),
    ("wagahaiwa_nekodearu.txt", "--model_type=bpe --vocab_size=4000 --normalization_rule_name=nfkc "
                                "--split_by_unicode_script=false --user_defined_symbols=<u>"),
])
def test_spm_train_bpe_matches_oracle(corpus, args, tmp_path):
    prefix, _ = _train_gpu(tmp_path, os.path.join(GOLD, corpus), args, "bp")
    _check_vs_oracle(prefix, args, _lines(corpus))


def test_spm_train_bpe_synthetic(tmp_path):
    """30k synthetic lines (c3 distribution), vocab 4000, identity."""
    path = _synth_file(tmp_path, 30_000, seed=3)
    args = "--model_type=bpe --vocab_size=4000 --normalization_rule_name=identity"
    prefix, _ = _train_gpu(tmp_path, path, args, "bsyn")
    _check_vs_oracle(prefix, args, O.read_lines_binary(path))


@pytest.mark.parametrize("corpus,args", [
    ("botchan.txt", "--model_type=bpe --vocab_size=2000 --normalization_rule_name=nfkc "
                    "--split_by_whitespace=false"),
    ("wagahaiwa_nekodearu.txt", "--model_type=bpe --vocab_size=4000 --normalization_rule_name=nfkc"),
    (None, "--model_type=bpe --vocab_size=3000 --normalization_rule_name=identity"),
])
def test_spm_train_bpe_device_refresh_checked(corpus, args, tmp_path):
    """The merge loop's pair-frequency refresh on the device
    (spm_hip_bpe_refresh: ComputeFreq of every reset bigram,
    bpe_model_trainer.cc:87-113, over device-resident symbol arrays and
    position sets): with SPM_HIP_BPE_REFRESH_CHECK=1 every refresh is
    recomputed on the host and any freq or erased-position difference fails
    the run; the model equals the oracle's and the host-refresh run's bytes.
    The runs of identical chars ("aaaa", "ーー") exercise the overlap rule.
    SPM_HIP_BPE_RELAYOUT_CHECK=1 also compares the symbol cache's walk before
    and after every relayout copy (the kept-set replay reads that order)."""
    if corpus is None:
        rng = np.random.default_rng(21)

        def word():
            return "".join("abcd"[int(rng.integers(0, 4))] * int(rng.integers(1, 6))
                           for _ in range(int(rng.integers(1, 5))))
        lines = [" ".join(word() for _ in range(8)) for _ in range(3000)]
        path = str(tmp_path / "runs.txt")
        open(path, "w").write("\n".join(lines) + "\n")
        lines_b = O.read_lines_binary(path)
    else:
        path = os.path.join(GOLD, corpus)
        lines_b = _lines(corpus)
    prefix, _ = _train_gpu(tmp_path, path, args + " --timings", "rc",
                           env={"SPM_HIP_BPE_REFRESH_CHECK": "1", "SPM_HIP_BPE_RELAYOUT_CHECK": "1"})
    tm = json.loads([l for l in _train_gpu.last_stdout.splitlines() if l.startswith("{")][-1])
    assert tm["bpe_refresh_checked"] == tm["bpe_updates"] > 0
    _check_vs_oracle(prefix, args, lines_b)
    hprefix, _ = _train_gpu(tmp_path, path, args, "rh", env={"SPM_HIP_BPE_DEVICE_REFRESH": "0"})
    # (the .model bytes differ in the serialized model_prefix; the pieces must not)
    assert (model_reader.read_pieces(open(prefix + ".model", "rb").read()) ==
            model_reader.read_pieces(open(hprefix + ".model", "rb").read()))
    assert open(prefix + ".vocab", "rb").read() == open(hprefix + ".vocab", "rb").read()


@pytest.mark.parametrize("model_type,extra", [
    ("unigram", ""),
    ("unigram", "--treat_whitespace_as_suffix=true"),
    ("bpe", ""),
])
def test_spm_train_device_split_equals_host_split(model_type, extra, tmp_path):
    """SplitSentencesByWhitespace on the device (split_kernels.hip: hash sort,
    byte-compared runs, summed freqs) trains the same model as the host split
    (--host_split=true, the device path's fallback): the same pieces, score
    bits, types and .vocab bytes, on a corpus with multi-byte chars, broken
    UTF-8 and repeated words."""
    rng = np.random.default_rng(17)
    alpha = list("abcdef") + ["ü", "日", "本", "語", "ÿ"]
    words = ["".join(alpha[int(x)] for x in rng.integers(0, len(alpha), int(rng.integers(1, 9))))
             for _ in range(200)]
    lines = []
    for _ in range(5000):
        k = int(rng.integers(1, 8))
        lines.append(" ".join(words[int(rng.integers(0, len(words)))] for _ in range(k)))
    raw = "\n".join(lines).encode() + b"\n\xe3\x81\n\xc3\n"
    path = tmp_path / "c.txt"
    path.write_bytes(raw)
    args = ("--model_type=%s --vocab_size=100 --normalization_rule_name=identity --num_threads=4 %s"
            % (model_type, extra))
    dev, _ = _train_gpu(tmp_path, str(path), args, "dev")
    assert "device split of" in _train_gpu.last_log
    host, _ = _train_gpu(tmp_path, str(path), args + " --host_split=true", "host")
    assert "host split" in _train_gpu.last_log
    # The device split's own fallback exit (a hash collision), forced after
    # all of its device work: the corpus comes back from HBM into the host
    # split (bytes, offsets, freqs kept).
    fb, _ = _train_gpu(tmp_path, str(path), args, "fallback", env={"SPM_HIP_SPLIT_FORCE_FALLBACK": "1"})
    assert "hash collision or size limit, host split" in _train_gpu.last_log
    # (the .model bytes also hold the TrainerSpec's model_prefix, which differs)
    got_d = model_reader.read_pieces(open(dev + ".model", "rb").read())
    for other in (host, fb):
        got_h = model_reader.read_pieces(open(other + ".model", "rb").read())
        assert [g[0] for g in got_d] == [g[0] for g in got_h]
        assert [g[2] for g in got_d] == [g[2] for g in got_h]
        assert np.array_equal(np.array([g[1] for g in got_d], dtype=np.float32).view(np.uint32),
                              np.array([g[1] for g in got_h], dtype=np.float32).view(np.uint32))
        assert open(dev + ".vocab", "rb").read() == open(other + ".vocab", "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("tail", [b"\n", b"", b"\n\n"])
def test_spm_train_device_load_equals_host_load(tail, tmp_path):
    """ReadCorpus's device path (the file copied to HBM, lines found and
    filtered by CorpusParseLines, SPM_HIP_DEVICE_LOAD=1) trains the same model
    as the host parse: empty lines, lines holding kUNKStr (U+2585), lines
    over max_sentence_length, CR bytes, NULs, multi-byte text, and a file
    ending with / without / with two newlines (std::getline semantics)."""
    rng = np.random.default_rng(5)
    alpha = list("abcdefgh") + ["ü", "日", "本"]
    lines = []
    for k in range(6000):
        w = " ".join("".join(alpha[int(x)] for x in rng.integers(0, len(alpha), int(rng.integers(1, 7))))
                     for _ in range(int(rng.integers(1, 6))))
        r = k % 97
        if r == 3:
            w = ""
        elif r == 5:
            w = w + " \u2585 " + w  # kUNKStr: the line is dropped
        elif r == 6:
            w = w + " \u2047 " + w
        elif r == 7:
            w = w * 40  # over --max_sentence_length=300
        elif r == 11:
            w = w + "\r"
        elif r == 13:
            w = w + "\x00x"
        lines.append(w.encode())
    raw = b"\n".join(lines) + tail
    path = tmp_path / "c.txt"
    path.write_bytes(raw)
    args = "--vocab_size=120 --normalization_rule_name=identity --num_threads=4 --max_sentence_length=300"
    dev, _ = _train_gpu(tmp_path, str(path), args, "dev", env={"SPM_HIP_DEVICE_LOAD": "1"})
    log_dev = _train_gpu.last_log
    host, _ = _train_gpu(tmp_path, str(path), args, "host", env={"SPM_HIP_DEVICE_LOAD": "0"})
    log_host = _train_gpu.last_log
    for pat in ("Loaded ", "too long sentences"):
        ld = [l for l in log_dev.splitlines() if pat in l]
        lh = [l for l in log_host.splitlines() if pat in l]
        assert ld == lh and ld, (pat, ld, lh)
    assert open(dev + ".vocab", "rb").read() == open(host + ".vocab", "rb").read()
    got_d = model_reader.read_pieces(open(dev + ".model", "rb").read())
    got_h = model_reader.read_pieces(open(host + ".model", "rb").read())
    assert got_d == got_h


@pytest.mark.parametrize("parts", [2, 4, 8])
@pytest.mark.parametrize("corpus,args", [SEED_CASES[0], SEED_CASES[1], SEED_CASES[3]])
def test_seed_mine_msd_parts(monkeypatch, parts, corpus, args):
    """The suffix order split by first-symbol ranges (the large-corpus
    layout: each part sorted on its own into its segment of SA, sort buffers
    of one part), forced on small corpora: seeds and scores identical to the
    literal esaxx restatement."""
    import spm_amd
    monkeypatch.setenv("SPM_HIP_SEED_PARTS", str(parts))
    ot = O.OracleTrainer(args, _lines(corpus), _charsmap(_rule_of(args)))
    sents, freq = ot.sentences()
    want_p, want_s = ot.seeds()
    cnt = collections.Counter()
    for s, f in zip(sents, freq):
        for ch in s.decode():
            if ch != "▅":
                cnt[ord(ch)] += int(f)
    chars = sorted(cnt)
    got_p, got_s, st = spm_amd.seed_mine(
        sents, chars, [cnt[c] for c in chars],
        max_sentencepiece_length=int(_flag(args, "max_sentencepiece_length", 16)),
        split_by_unicode_script=_flag(args, "split_by_unicode_script", "true") == "true",
        split_by_number=_flag(args, "split_by_number", "true") == "true",
        split_by_whitespace=_flag(args, "split_by_whitespace", "true") == "true",
        treat_whitespace_as_suffix=_flag(args, "treat_whitespace_as_suffix", "false") == "true",
        seed_sentencepiece_size=int(_flag(args, "seed_sentencepiece_size", 1000000)))
    assert got_p == want_p
    assert np.array_equal(got_s.view(np.uint32), want_s.view(np.uint32))


def test_seed_mine_node_capacity_rerun(monkeypatch):
    """The candidate nodes are first written into buffers the suffix sort
    no longer needs (room for N/2); a corpus with more candidates re-runs
    the node kernel with exact room.  Forced here with a capacity of 16:
    seeds and scores stay identical to the literal esaxx restatement."""
    import spm_amd
    monkeypatch.setenv("SPM_HIP_SEED_NODE_CAP", "16")
    args = "--vocab_size=1000 --normalization_rule_name=nfkc"
    ot = O.OracleTrainer(args, _lines("botchan.txt"), _charsmap("nfkc"))
    sents, freq = ot.sentences()
    want_p, want_s = ot.seeds()
    cnt = collections.Counter()
    for s, f in zip(sents, freq):
        for ch in s.decode():
            if ch != "▅":
                cnt[ord(ch)] += int(f)
    chars = sorted(cnt)
    got_p, got_s, st = spm_amd.seed_mine(sents, chars, [cnt[c] for c in chars])
    assert got_p == want_p
    assert np.array_equal(got_s.view(np.uint32), want_s.view(np.uint32))
