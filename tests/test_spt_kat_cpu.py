"""The reference's own known answers for norm_to_orig (NormalizeFullTest,
normalizer_test.cc:321-401) and SentencePieceText (EncodeTest,
sentencepiece_processor_test.cc:129-240) on the CPU oracle; the same
vectors run through the device path in tests/test_gpu_spt.py."""
import oracle_lib as O
import spt_known_answers as KA


def test_oracle_normalize_full_test():
    om = O.OracleModel(KA.normalizer_model())
    got = om.normalize_align([i.encode() for i, _, _ in KA.NORMALIZE_FULL])
    for (inp, want, n2i), (norm, a) in zip(KA.NORMALIZE_FULL, got):
        assert norm == want.encode(), inp
        assert a == n2i, inp


def test_oracle_encode_test_spt():
    for name, pieces, rows in KA.ENCODE_CASES:
        om = O.OracleModel(KA.encode_model(pieces))
        om.set_extra_options("eos")
        got = om.encode_spt([KA.ENCODE_INPUT])[0]
        assert got == [(i, p.encode(), s.encode(), b, e) for i, p, s, b, e in rows], name
