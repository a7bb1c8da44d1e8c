"""CPU tests of the unigram trainer path (spm_train): the oracle against the
reference's own known-answer test, the Unicode script table against the
reference's table, and oracle invariants.  No GPU."""
import os

import numpy as np
import pytest

import model_builder as mb
import oracle_lib
import script_table

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
WS = "▁"

# unigram_model_trainer_test.cc:47-86 (EndToEndTest)
KAT_ARGS = ("--vocab_size=8000 --normalization_rule_name=identity --model_type=unigram "
            "--user_defined_symbols=<user> --control_symbols=<ctrl> --max_sentence_length=2048")
KAT_TEXT = ("吾輩《わがはい》は猫である。名前はまだ無い。"
            "どこで生れたかとんと見当《けんとう》がつかぬ。"
            "何でも薄暗いじめじめした所でニャーニャー泣いていた事だけは記憶している。")
KAT_WANT = (WS + " 吾輩 《 わが はい 》 は 猫 である 。 名前 はまだ 無い 。 "
            "どこ で 生 れた か とん と 見当 《 けん とう 》 が つか ぬ 。 "
            "何でも 薄 暗 い じめ じめ した 所で ニャーニャー "
            "泣 い ていた 事 だけは 記憶 している 。")


def wagahaiwa_lines():
    return oracle_lib.read_lines_binary(os.path.join(GOLD, "wagahaiwa_nekodearu.txt"))


@pytest.mark.skipif(not os.path.exists(script_table.REF_MAP), reason="reference tree absent")
def test_script_table_matches_reference_map():
    bad = script_table.mismatches(script_table.load_table(), script_table.load_reference_map())
    assert bad == [], bad[:10]


def encode_with(pieces, scores, types, text):
    m = mb.model([(a, float(b), int(c)) for a, b, c in zip(pieces, scores, types)])
    om = oracle_lib.OracleModel(m)
    ids = om.encode_lines([text.encode()])[0]
    return " ".join(pieces[i].decode() for i in ids)


def test_oracle_train_known_answer():
    t = oracle_lib.OracleTrainer(KAT_ARGS, wagahaiwa_lines())
    p, s, ty = t.train()
    assert len(p) == 8000
    # <unk> <s> </s> then <ctrl> (CONTROL) and <user> (USER_DEFINED).
    assert [x.decode() for x in p[:5]] == ["<unk>", "<s>", "</s>", "<ctrl>", "<user>"]
    assert list(ty[:5]) == [mb.UNKNOWN, mb.CONTROL, mb.CONTROL, mb.CONTROL, mb.USER_DEFINED]
    assert encode_with(p, s, ty, "") == ""
    assert encode_with(p, s, ty, KAT_TEXT) == KAT_WANT
    # Scores after the meta pieces are non-increasing (Sorted in Finalize).
    assert np.all(np.diff(s[5:]) <= 0)


def test_oracle_seed_invariants():
    t = oracle_lib.OracleTrainer(KAT_ARGS, wagahaiwa_lines())
    sents, freq = t.sentences()
    seeds, scores = t.seeds()
    assert len(set(seeds)) == len(seeds)
    chars = set()
    for s in sents:
        chars.update(s.decode())
    chars.discard("▅")
    nchar = sum(1 for x in seeds if len(x.decode()) == 1)
    assert nchar == len(chars)
    # ToLogProb: log-probabilities whose float sum of exp is ~1.
    assert abs(np.exp(scores.astype(np.float64)).sum() - 1.0) < 1e-3
    for x in seeds[nchar:]:
        u = x.decode()
        assert 2 <= len(u) <= 16 and "▅" not in u and WS not in u[1:]


# bpe_model_trainer_test.cc:26-91 (BasicTest: vocab_size = size - 3,
# identity, no dummy prefix; pieces from id 3 on)
BPE_BASIC = [
    (["abracadabra"], 20, [], "ab ra abra ad cad abracad abracadabra ac br a b r c d"),
    (["pen", "pineapple", "apple"], 20, [], "ap le app apple en in ine pen p e a l n i"),
    (["hellohe"], 20, [], "he ll llo hello hellohe el lo oh hel ohe e h l o"),
    (["pen", "pineapple", "apple"], 20, ["app"], "app le en in ine pen pine ne pe e l n p i"),
]
BPE_KAT_ARGS = ("--vocab_size=8000 --normalization_rule_name=identity --model_type=bpe "
                "--control_symbols=<ctrl> --max_sentence_length=2048")
# bpe_model_trainer_test.cc:93-126 (EndToEndTest)
BPE_KAT_WANT = (WS + " 吾輩 《 わが はい 》 は猫 である 。 名前 はまだ 無い 。 "
                "どこで 生 れた か とん と見 当 《 けんとう 》 が つかぬ 。 "
                "何でも 薄 暗 いじ め じ め した 所で ニャー ニャー 泣 いていた "
                "事 だけは 記憶 している 。")


def bpe_basic_args(size, uds):
    a = "--model_type=bpe --vocab_size=%d --normalization_rule_name=identity --add_dummy_prefix=false" % (size - 3)
    return a + (" --user_defined_symbols=" + ",".join(uds) if uds else "")


@pytest.mark.parametrize("lines,size,uds,want", BPE_BASIC)
def test_oracle_bpe_train_basic(lines, size, uds, want):
    t = oracle_lib.OracleTrainer(bpe_basic_args(size, uds), [l.encode() for l in lines])
    p, s, ty = t.train()
    assert " ".join(x.decode() for x in p[3:]) == want


def test_oracle_bpe_train_known_answer():
    t = oracle_lib.OracleTrainer(BPE_KAT_ARGS, wagahaiwa_lines())
    p, s, ty = t.train()
    assert len(p) == 8000
    assert [x.decode() for x in p[:4]] == ["<unk>", "<s>", "</s>", "<ctrl>"]
    assert list(ty[:4]) == [mb.UNKNOWN, mb.CONTROL, mb.CONTROL, mb.CONTROL]
    m = mb.model([(a, float(b), int(c)) for a, b, c in zip(p, s, ty)], mb.BPE)
    om = oracle_lib.OracleModel(m)
    assert om.encode_lines([b""])[0] == []
    ids = om.encode_lines([KAT_TEXT.encode()])[0]
    assert " ".join(p[i].decode() for i in ids) == BPE_KAT_WANT
    # BPE scores are -merge rank (bpe_model_trainer.cc:269)
    assert np.array_equal(s[4:], -np.arange(len(p) - 4, dtype=np.float32))
