"""Seeded synthetic corpus for the encode/E-step benchmarks.

* 60,000 distinct pseudo-words over [a-z], length uniform in 2..10, drawn with
  random.Random(1234), shuffled (rank order = shuffled order).
* Sentences: word ranks drawn from Zipf p ∝ r^-1.1 with
  numpy.default_rng(seed); words are appended (single spaces) while the
  sentence is shorter than STOP_LEN characters.  STOP_LEN = 22 gives a mean of
  ≈25 raw characters per sentence (see DESIGN.md for the measured mean).

`normalized(...)` emits the bytes the reference normalizer produces for these
lines under nmt_nfkc / nfkc / identity with the default
add_dummy_prefix / remove_extra_whitespaces / escape_whitespaces flags:
"▁" + words joined by "▁" (normalizer.cc:88-211).  tests check this claim
against the host normalizer on a sample.
"""
import random

import numpy as np

NUM_WORDS = 60000
STOP_LEN = 22
WS = "▁".encode()


def make_words(seed=1234):
    r = random.Random(seed)
    seen = set()
    words = []
    while len(words) < NUM_WORDS:
        n = r.randint(2, 10)
        w = "".join(chr(97 + r.randrange(26)) for _ in range(n))
        if w not in seen:
            seen.add(w)
            words.append(w)
    r.shuffle(words)
    return words


_WORDS = None


def _word_table():
    global _WORDS
    if _WORDS is None:
        words = make_words()
        lens = np.array([len(w) for w in words], dtype=np.int64)
        tab = np.zeros((len(words), 10), dtype=np.uint8)
        for i, w in enumerate(words):
            tab[i, :len(w)] = np.frombuffer(w.encode(), dtype=np.uint8)
        p = np.arange(1, len(words) + 1, dtype=np.float64) ** -1.1
        cdf = np.cumsum(p / p.sum())
        cdf[-1] = 1.0
        _WORDS = (words, lens, tab, cdf)
    return _WORDS


def _draw(n, seed):
    """Returns (flat word ranks in sentence order, words per sentence)."""
    words, lens, tab, cdf = _word_table()
    rng = np.random.default_rng(seed)
    cur = np.zeros(n, dtype=np.int64)      # current char length
    nw = np.zeros(n, dtype=np.int64)
    cols = []
    active = np.arange(n)
    while active.size:
        r = np.searchsorted(cdf, rng.random(active.size), side="right")
        r = np.minimum(r, len(words) - 1)
        col = np.full(n, -1, dtype=np.int64)
        col[active] = r
        cols.append(col)
        add = lens[r] + (nw[active] > 0)
        cur[active] += add
        nw[active] += 1
        active = active[cur[active] < STOP_LEN]
    mat = np.stack(cols, axis=1)            # [n, maxw], -1 padded
    flat = mat[mat >= 0]                    # row-major = sentence order
    return flat, nw


def _emit(flat, nw, sep, prefix):
    """Builds a CSR byte buffer: prefix + w0 + sep + w1 ... per sentence."""
    words, lens, tab, cdf = _word_table()
    n = nw.size
    wl = lens[flat]
    first = np.zeros(flat.size, dtype=bool)
    starts = np.concatenate([[0], np.cumsum(nw)[:-1]])
    first[starts] = True
    lead = np.where(first, len(prefix), len(sep))
    piece_len = wl + lead
    total = int(piece_len.sum())
    out = np.empty(total, dtype=np.uint8)
    pstart = np.concatenate([[0], np.cumsum(piece_len)[:-1]])
    # separators / prefixes
    for k in range(max(len(prefix), len(sep))):
        if k < len(sep):
            m = (~first)
            out[pstart[m] + k] = sep[k]
        if k < len(prefix):
            m = first
            out[pstart[m] + k] = prefix[k]
    # word chars
    wstart = pstart + lead
    for c in range(10):
        m = wl > c
        out[wstart[m] + c] = tab[flat[m], c]
    sent_len = np.add.reduceat(piece_len, starts) if n else np.zeros(0, np.int64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(sent_len)
    return out, off


def raw(n, seed=1234):
    """Raw lines as a CSR (bytes uint8, offsets uint64[n+1])."""
    flat, nw = _draw(n, seed)
    return _emit(flat, nw, b" ", b"")


def normalized(n, seed=1234):
    """Normalized sentences ("▁w0▁w1...") as a CSR."""
    flat, nw = _draw(n, seed)
    return _emit(flat, nw, WS, WS)


def lines(n, seed=1234):
    buf, off = raw(n, seed)
    b = buf.tobytes()
    return [b[int(off[i]):int(off[i + 1])] for i in range(n)]
