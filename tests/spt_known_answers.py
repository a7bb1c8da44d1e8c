"""Known answers for norm_to_orig and SentencePieceText, restated from the
reference's own unit tests (test infrastructure).

* NormalizeFullTest (src/normalizer_test.cc:321-401): Normalizer::Normalize
  with the nmt_nfkc NormalizerSpec (MakeDefaultSpec, :38-40): the normalized
  string and the exact n2i (norm_to_orig) vector of five inputs.  The
  charsmap is data/normalization/nmt_nfkc.bin (the blob embedded in
  data/synth32k_unigram.model: pip sentencepiece 0.2.2's nmt_nfkc, a
  substitute for the reference-era blob); every mapping these
  five inputs exercise (fullwidth space, halfwidth katakana, circled digits,
  ㍿) is plain NFKC.
* SentencepieceProcessorTest.EncodeTest (src/sentencepiece_processor_test.cc:
  129-240): SentencePieceProcessor::Encode("ABC DEF", SentencePieceText*)
  with a MockModel whose Encode returns fixed pieces.  Here the MockModel
  results become hand-built unigram models whose Viterbi yields the same
  pieces and ids ({▁ABC: 3, ▁DE: 4} and {▁ABC: 3, ▁D: 4}; F, E and F are
  out of vocabulary, hence UNKNOWN id 0, and E F merge into one piece).  The
  mock's trailing "</s>" (id 2) comes out of ModelInterface::Encode itself,
  which a real model never does (CONTROL pieces live in reserved_id_map_,
  outside the trie, model_interface.cc:101-144); the `eos` extra option adds
  the same piece through ApplyExtraOptions (sentencepiece_processor.cc:
  953-959), which sets only id and piece, so its begin/end stay 0.
"""
import os

from model_builder import CONTROL, NORMAL, UNKNOWN, UNIGRAM, model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WS = "▁"


def nmt_nfkc():
    return open(os.path.join(ROOT, "data", "normalization", "nmt_nfkc.bin"), "rb").read()


# (input, expected normalized, expected n2i) — normalizer_test.cc:327-400.
NORMALIZE_FULL = [
    ("I saw a girl", WS + "I" + WS + "saw" + WS + "a" + WS + "girl",
     [0, 0, 0, 0, 1, 1, 1, 2, 3, 4, 5, 5, 5, 6, 7, 7, 7, 8, 9, 10, 11, 12]),
    (" I   saw a　 　girl　　", WS + "I" + WS + "saw" + WS + "a" + WS + "girl",
     [1, 1, 1, 1, 2, 2, 2, 5, 6, 7, 8, 8, 8, 9, 10, 10, 10, 17, 18, 19, 20, 21]),
    (" ｸﾞｰｸﾞﾙ ", WS + "グーグル",
     [1, 1, 1, 1, 1, 1, 7, 7, 7, 10, 10, 10, 16, 16, 16, 19]),
    ("①②③", WS + "123", [0, 0, 0, 0, 3, 6, 9]),
    ("㍿", WS + "株式会社", [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 3]),
]


def normalizer_model():
    """Default NormalizerSpec (add_dummy_prefix, remove_extra_whitespaces,
    escape_whitespaces) with the nmt_nfkc charsmap; the pieces are
    irrelevant to normalization."""
    pieces = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL), (WS, -1.0, NORMAL)]
    return model(pieces, UNIGRAM, charsmap=nmt_nfkc())


# EncodeTest (sentencepiece_processor_test.cc:129-240): the model's pieces
# and the expected (id, piece, surface, begin, end) rows of
# Encode("ABC DEF", &spt) with the `eos` extra option.
ENCODE_CASES = [
    ("encode", [(WS + "ABC", -1.0), (WS + "DE", -1.0)],
     [(3, WS + "ABC", "ABC", 0, 3), (4, WS + "DE", " DE", 3, 6), (0, "F", "F", 6, 7), (2, "</s>", "", 0, 0)]),
    ("unknown_sequence", [(WS + "ABC", -1.0), (WS + "D", -1.0)],
     [(3, WS + "ABC", "ABC", 0, 3), (4, WS + "D", " D", 3, 5), (0, "EF", "EF", 5, 7), (2, "</s>", "", 0, 0)]),
]
ENCODE_INPUT = b"ABC DEF"


def encode_model(pieces):
    base = [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL)]
    return model(base + [(p, s, NORMAL) for p, s in pieces], UNIGRAM, charsmap=nmt_nfkc())
