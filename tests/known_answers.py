"""Known-answer cases restated from the reference's own unit tests.

Each case: (name, model bytes, [(normalized input, expected pieces)]).
Sources: src/unigram_model_test.cc:222-241 (LatticeTest.ViterbiTest, as
models whose trie yields the same lattice), :471-550 (PopulateNodes*),
:580-728 (EncodeTest, EncodeWithUnusedTest), src/bpe_model_test.cc:49-255 (EncodeTest, EncodeAmbiguous,
EncodeWithUnused).  The expected piece strings are copied from the EXPECT_EQ
lines of those tests.
"""
from model_builder import BPE, NORMAL, UNIGRAM, UNUSED, USER_DEFINED, base_pieces, model


def _encode_test_pieces():
    p = [("ab", 0.0), ("cd", -0.1), ("abc", -0.2), ("a", -0.3), ("b", -0.4), ("c", -0.5),
         ("ABC", -0.5), ("abcdabcd", -0.5), ("q", -0.5), ("r", -0.5), ("qr", -0.5)]
    ud = {"ABC", "abcdabcd", "q", "r"}
    return base_pieces() + [(s, sc, USER_DEFINED if s in ud else NORMAL) for s, sc in p]


_ENCODE_EXPECT = [
    ("abc", ["abc"]), ("AB", ["A", "B"]), ("abcd", ["ab", "cd"]), ("abcc", ["abc", "c"]),
    ("xabcabaabcdd", ["x", "abc", "ab", "a", "ab", "cd", "d"]),
    ("xyz東京", ["x", "y", "z", "東", "京"]), ("ABC", ["ABC"]), ("abABCcd", ["ab", "ABC", "cd"]),
    ("ababcdabcdcd", ["ab", "abcdabcd", "cd"]), ("abqrcd", ["ab", "q", "r", "cd"]), ("", []),
]


def _unused_pieces(unused, normal=()):
    p = [("abcd", 10.0), ("abc", 5.0), ("ab", 2.0), ("cd", 1.0), ("a", 0.0), ("b", 0.0),
         ("c", 0.0), ("d", 0.0)]
    out = base_pieces()
    for i, (s, sc) in enumerate(p):
        idx = i + 3
        out.append((s, sc, UNUSED if idx in unused else NORMAL))
    return out


def cases():
    c = []
    c.append(("unigram_encode", model(_encode_test_pieces(), UNIGRAM), _ENCODE_EXPECT))
    c.append(("bpe_encode", model(_encode_test_pieces(), BPE), _ENCODE_EXPECT))
    # EncodeWithUnusedTest (unigram_model_test.cc:675-728)
    c.append(("unigram_unused_0", model(_unused_pieces(set()), UNIGRAM), [("abcd", ["abcd"])]))
    c.append(("unigram_unused_3", model(_unused_pieces({3}), UNIGRAM), [("abcd", ["abc", "d"])]))
    c.append(("unigram_unused_35", model(_unused_pieces({3, 5}), UNIGRAM), [("abcd", ["abc", "d"])]))
    c.append(("unigram_unused_34", model(_unused_pieces({3, 4}), UNIGRAM), [("abcd", ["ab", "cd"])]))
    # bpe_model_test.cc:200-255
    c.append(("bpe_unused_0", model(_unused_pieces(set()), BPE), [("abcd", ["abcd"])]))
    c.append(("bpe_unused_3", model(_unused_pieces({3}), BPE), [("abcd", ["abc", "d"])]))
    c.append(("bpe_unused_35", model(_unused_pieces({3, 5}), BPE), [("abcd", ["abc", "d"])]))
    c.append(("bpe_unused_34", model(_unused_pieces({3, 4}), BPE), [("abcd", ["ab", "c", "d"])]))
    # EncodeAmbiguousTest (bpe_model_test.cc:145-190)
    amb = base_pieces() + [("aa", -0.1, NORMAL), ("bb", -0.2, NORMAL), ("ab", -0.3, NORMAL),
                           ("a", -0.4, NORMAL), ("b", -0.5, NORMAL)]
    c.append(("bpe_ambiguous", model(amb, BPE),
              [("aaa", ["aa", "a"]), ("aabb", ["aa", "bb"]), ("aaabbb", ["aa", "a", "bb", "b"]),
               ("aaaba", ["aa", "ab", "a"]), ("あ".encode()[:1], ["あ".encode()[:1]])]))
    # PopulateNodesAllUnknownsTest (unigram_model_test.cc:471-488): every node UNK.
    c.append(("unigram_all_unknown", model(base_pieces() + [("x", 0.0, NORMAL)], UNIGRAM),
              [("abc", ["a", "b", "c"])]))
    # PopulateNodesTest (:490-520) lattice; best path a(0.1)+bc(0.4) beats ab+UNK.
    pn = base_pieces() + [("a", 0.1, NORMAL), ("b", 0.2, NORMAL), ("ab", 0.3, NORMAL), ("bc", 0.4, NORMAL)]
    c.append(("unigram_populate", model(pn, UNIGRAM), [("abc", ["a", "bc"])]))
    # PopulateNodesWithUnusedTest (:522-548): ab / bc UNUSED never become nodes.
    pu = base_pieces() + [("a", 0.1, NORMAL), ("b", 0.2, NORMAL), ("ab", 0.3, UNUSED),
                          ("bc", 0.4, UNUSED)]
    c.append(("unigram_populate_unused", model(pu, UNIGRAM), [("abc", ["a", "b", "c"])]))
    # LatticeTest.ViterbiTest (:222-241): nodes inserted one by one with fixed
    # scores; here each stage is a model whose PopulateNodes builds that lattice.
    stages = [("A", 0.0), ("B", 0.0), ("C", 0.0)]
    for k, (extra, want) in enumerate([(None, ["A", "B", "C"]), (("AB", 2.0), ["AB", "C"]),
                                       (("BC", 5.0), ["A", "BC"]), (("ABC", 10.0), ["ABC"])]):
        if extra:
            stages.append(extra)
        c.append(("lattice_viterbi_%d" % k,
                  model(base_pieces() + [(p, s_, NORMAL) for p, s_ in stages], UNIGRAM),
                  [("ABC", want)]))
    return c


def populate_marginal_case():
    """LatticeTest.PopulateMarginalTest (unigram_model_test.cc:271-315) as an
    E-step: the TrainerModel piece list A, B, C, AB, BC, ABC (ids 0..5, the
    test's scores) over the sentence "ABC" with freq 1 builds exactly the
    test's lattice (every char has a 1-char piece, so no UNK node).  Returns
    (pieces, scores, sentence, expected marginals, log Z, Viterbi size); the
    reference checks marginals and log Z to 1e-3."""
    import math
    pieces = [b"A", b"B", b"C", b"AB", b"BC", b"ABC"]
    scores = [1.0, 1.2, 2.5, 3.0, 4.0, 2.0]
    p1 = math.exp(1.0 + 1.2 + 2.5)
    p2 = math.exp(3.0 + 2.5)
    p3 = math.exp(1.0 + 4.0)
    p4 = math.exp(2.0)
    Z = p1 + p2 + p3 + p4
    marg = [(p1 + p3) / Z, p1 / Z, (p1 + p2) / Z, p2 / Z, p3 / Z, p4 / Z]
    # Viterbi: AB C (5.5) beats A BC (5.0), A B C (4.7), ABC (2.0).
    return pieces, scores, b"ABC", marg, math.log(Z), 2


def as_bytes(x):
    return x if isinstance(x, bytes) else x.encode()


def split_pieces(inp, lens):
    out, k = [], 0
    b = as_bytes(inp)
    for n in lens:
        out.append(b[k:k + n])
        k += n
    return out
