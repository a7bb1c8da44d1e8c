"""Tiny ModelProto writer for hand-built test models (test infrastructure).

Mirrors the fixtures of the reference tests (MakeBaseModelProto / AddPiece in
unigram_model_test.cc:361-392, bpe_model_test.cc, sentencepiece_processor_test.cc).
Wire format of src/sentencepiece_model.proto.
"""
import struct

NORMAL, UNKNOWN, CONTROL, USER_DEFINED, UNUSED = 1, 2, 3, 4, 5
UNIGRAM, BPE = 1, 2


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wt):
    return _varint((field << 3) | wt)


def _ld(field, payload):
    return _key(field, 2) + _varint(len(payload)) + payload


def piece(s, score=0.0, type_=NORMAL):
    if isinstance(s, str):
        s = s.encode()
    body = _ld(1, s) + _key(2, 5) + struct.pack("<f", score)
    if type_ != NORMAL:
        body += _key(3, 0) + _varint(type_)
    return body


def model(pieces, model_type=UNIGRAM, charsmap=b"", add_dummy_prefix=True,
          remove_extra_whitespaces=True, escape_whitespaces=True, treat_ws_as_suffix=False):
    """pieces: list of (str|bytes, score, type)."""
    out = b"".join(_ld(1, piece(*p)) for p in pieces)
    ts = _key(3, 0) + _varint(model_type)
    if treat_ws_as_suffix:
        ts += _key(24, 0) + _varint(1)
    out += _ld(2, ts)
    ns = b""
    if charsmap:
        ns += _ld(2, charsmap)
    ns += _key(3, 0) + _varint(int(add_dummy_prefix))
    ns += _key(4, 0) + _varint(int(remove_extra_whitespaces))
    ns += _key(5, 0) + _varint(int(escape_whitespaces))
    out += _ld(3, ns)
    return out


def base_pieces():
    """MakeBaseModelProto: <unk>, <s>, </s> (unigram_model_test.cc:361-378)."""
    return [("<unk>", 0.0, UNKNOWN), ("<s>", 0.0, CONTROL), ("</s>", 0.0, CONTROL)]
