"""Reads (piece, score, type) from a serialized ModelProto (test helper)."""
import struct


def _varint(b, i):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        if not c & 0x80:
            return v, i
        s += 7


def _fields(b):
    i = 0
    while i < len(b):
        k, i = _varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 2:
            n, i = _varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            raise ValueError("bad wire type")
        yield f, wt, v


def read_pieces(model_bytes):
    out = []
    for f, wt, v in _fields(model_bytes):
        if f == 1 and wt == 2:
            p, s, t = b"", 0.0, 1
            for g, gt, w in _fields(v):
                if g == 1:
                    p = bytes(w)
                elif g == 2:
                    s = struct.unpack("<f", w)[0]
                elif g == 3:
                    t = w if 1 <= w <= 5 else 1
            out.append((p, s, t))
    return out


def fields(model_bytes):
    """(field, wire type, value) of the top-level message."""
    return list(_fields(model_bytes))


def sub_fields(msg_bytes):
    return list(_fields(msg_bytes))


def charsmap(model_bytes):
    """NormalizerSpec.precompiled_charsmap of a ModelProto (b"" if none)."""
    for f, wt, v in _fields(model_bytes):
        if f == 3 and wt == 2:
            for g, gt, w in _fields(v):
                if g == 2:
                    return bytes(w)
    return b""
