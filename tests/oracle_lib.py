"""ctypes binding of the CPU oracle (oracle/_build/libspm_oracle.so).

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  Builds the oracle on first use if needed.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "libspm_oracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "spm_oracle.cc")
        if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_load.restype = P
        L.oracle_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_free.argtypes = [P]
        L.oracle_model_type.argtypes = [P]
        L.oracle_piece_size.argtypes = [P]
        L.oracle_set_extra_options.argtypes = [P, ctypes.c_char_p]
        L.oracle_normalize_batch.argtypes = [P, P, P, ctypes.c_uint64, P, P]
        L.oracle_encode_normalized_batch.argtypes = [P, P, P, ctypes.c_uint64, P, P, P, ctypes.c_int]
        L.oracle_encode_lines.argtypes = [P, P, P, ctypes.c_uint64, P, P]
        L.oracle_normalize_align.argtypes = [P, P, P, ctypes.c_uint64, P, P, P, P]
        L.oracle_encode_spt_lines.argtypes = [P, P, P, ctypes.c_uint64, P, P, P, P, P, P]
        L.oracle_estep.argtypes = [P, P, P, ctypes.c_uint64, P, P, P, ctypes.c_uint64,
                                   ctypes.c_int, P, P, P]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def to_csr(items):
    """list[bytes] -> (uint8 buffer, uint64 offsets[n+1])."""
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    buf = np.frombuffer(b"".join(items), dtype=np.uint8).copy()
    if buf.size == 0:
        buf = np.zeros(1, dtype=np.uint8)
    return buf, off


def from_csr(vals, off):
    return [vals[int(off[i]):int(off[i + 1])].tolist() for i in range(len(off) - 1)]


class OracleModel:
    def __init__(self, model_bytes):
        self.L = lib()
        self._bytes = bytes(model_bytes)
        self.h = self.L.oracle_load(self._bytes, len(self._bytes))
        if not self.h:
            raise ValueError("oracle: cannot load model")

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_free(self.h)
            self.h = None

    @property
    def model_type(self):
        return self.L.oracle_model_type(self.h)

    def set_extra_options(self, s):
        rc = self.L.oracle_set_extra_options(self.h, s.encode())
        if rc:
            raise ValueError("bad extra option")

    def normalize(self, lines):
        buf, off = to_csr(lines)
        cap = int(off[-1]) * 3 + 4 * len(lines) + 16
        out = np.zeros(cap, dtype=np.uint8)
        oo = np.zeros(len(lines) + 1, dtype=np.uint64)
        self.L.oracle_normalize_batch(self.h, _ptr(buf), _ptr(off), len(lines), _ptr(out), _ptr(oo))
        return [out[int(oo[i]):int(oo[i + 1])].tobytes() for i in range(len(lines))]

    def normalize_align(self, lines):
        """[(normalized bytes, norm_to_orig list)] (the reference's vector: empty
        for empty / all-whitespace input)."""
        buf, off = to_csr(lines)
        cap = int(off[-1]) * 3 + 4 * len(lines) + 16
        out = np.zeros(cap, dtype=np.uint8)
        oo = np.zeros(len(lines) + 1, dtype=np.uint64)
        a = np.zeros(cap + len(lines) + 16, dtype=np.uint64)
        ao = np.zeros(len(lines) + 1, dtype=np.uint64)
        self.L.oracle_normalize_align(self.h, _ptr(buf), _ptr(off), len(lines), _ptr(out), _ptr(oo),
                                      _ptr(a), _ptr(ao))
        return [(out[int(oo[i]):int(oo[i + 1])].tobytes(), a[int(ao[i]):int(ao[i + 1])].tolist())
                for i in range(len(lines))]

    def encode_spt(self, lines):
        """Encode(SentencePieceText) per line: [(id, piece, surface, begin, end)]."""
        buf, off = to_csr(lines)
        cap = int(off[-1]) * 3 + 4 * len(lines) + 64 * len(lines) + 16
        rec = np.zeros(3 * cap, dtype=np.int64)
        po = np.zeros(len(lines) + 1, dtype=np.uint64)
        ps = np.zeros(cap * 4 + 1024, dtype=np.uint8)
        pso = np.zeros(cap + 1, dtype=np.uint64)
        ss = np.zeros(cap * 4 + 1024, dtype=np.uint8)
        sso = np.zeros(cap + 1, dtype=np.uint64)
        rc = self.L.oracle_encode_spt_lines(self.h, _ptr(buf), _ptr(off), len(lines), _ptr(rec), _ptr(po),
                                            _ptr(ps), _ptr(pso), _ptr(ss), _ptr(sso))
        if rc:
            raise RuntimeError("oracle encode_spt failed: %d" % rc)
        out = []
        for i in range(len(lines)):
            row = []
            for k in range(int(po[i]), int(po[i + 1])):
                row.append((int(rec[3 * k]), ps[int(pso[k]):int(pso[k + 1])].tobytes(),
                            ss[int(sso[k]):int(sso[k + 1])].tobytes(), int(rec[3 * k + 1]),
                            int(rec[3 * k + 2])))
            out.append(row)
        return out

    def encode_normalized_csr(self, buf, off, threads=1, with_lens=False):
        n = len(off) - 1
        cap = max(int(off[-1]), 1)
        ids = np.zeros(cap, dtype=np.int32)
        lens = np.zeros(cap, dtype=np.uint32) if with_lens else None
        to = np.zeros(n + 1, dtype=np.uint64)
        self.L.oracle_encode_normalized_batch(self.h, _ptr(buf), _ptr(off), n, _ptr(ids),
                                              _ptr(lens) if with_lens else None, _ptr(to), threads)
        if with_lens:
            return ids[:int(to[-1])], lens[:int(to[-1])], to
        return ids[:int(to[-1])], to

    def encode_normalized(self, sentences, threads=1):
        buf, off = to_csr(sentences)
        ids, to = self.encode_normalized_csr(buf, off, threads)
        return from_csr(ids, to)

    def encode_lines(self, lines):
        buf, off = to_csr(lines)
        cap = int(off[-1]) * 3 + 6 * len(lines) + 16
        ids = np.zeros(cap, dtype=np.int32)
        to = np.zeros(len(lines) + 1, dtype=np.uint64)
        rc = self.L.oracle_encode_lines(self.h, _ptr(buf), _ptr(off), len(lines), _ptr(ids), _ptr(to))
        if rc:
            raise RuntimeError("oracle encode failed: %d" % rc)
        return from_csr(ids, to)


def estep(sentences, freqs, pieces, scores, threads):
    """RunEStep emulation.  Returns (expected float32[V], obj float, ntok int)."""
    L = lib()
    sb, so = to_csr(sentences)
    pb, po = to_csr(pieces)
    fr = np.asarray(freqs, dtype=np.int64)
    sc = np.asarray(scores, dtype=np.float32)
    V = len(pieces)
    exp = np.zeros(V, dtype=np.float32)
    obj = np.zeros(1, dtype=np.float32)
    nt = np.zeros(1, dtype=np.int64)
    L.oracle_estep(_ptr(sb), _ptr(so), _ptr(fr), len(sentences), _ptr(pb), _ptr(po), _ptr(sc), V,
                   threads, _ptr(exp), _ptr(obj), _ptr(nt))
    return exp, float(obj[0]), int(nt[0])


def estep_cyclic_csr(buf, off, freqs, n_total, pieces, scores, threads):
    """RunEStep emulation over sentence g = buffer[g mod n], g < n_total (the
    bench's re-used resident buffer).  buf/off: CSR of the n buffer sentences."""
    L = lib()
    if not hasattr(L, "_cyclic_bound"):
        P = ctypes.c_void_p
        L.oracle_estep_cyclic.argtypes = [P, P, P, ctypes.c_uint64, ctypes.c_uint64, P, P, P, ctypes.c_uint64,
                                          ctypes.c_int, P, P, P]
        L._cyclic_bound = True
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    pb, po = to_csr(pieces)
    fr = np.ascontiguousarray(freqs, dtype=np.int64)
    sc = np.ascontiguousarray(scores, dtype=np.float32)
    V = len(pieces)
    exp = np.zeros(V, dtype=np.float32)
    obj = np.zeros(1, dtype=np.float32)
    nt = np.zeros(1, dtype=np.int64)
    L.oracle_estep_cyclic(_ptr(buf), _ptr(off), _ptr(fr), len(off) - 1, int(n_total), _ptr(pb), _ptr(po), _ptr(sc),
                          V, threads, _ptr(exp), _ptr(obj), _ptr(nt))
    return exp, float(obj[0]), int(nt[0])


def read_lines_binary(path):
    data = open(path, "rb").read()
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    return lines


def estep_partial(sentences, freqs, pieces, scores, all_freq, mode, T, index_base, index_stride,
                  acc, acc_obj, ntok_acc):
    """oracle_estep_partial into numpy accumulators (see dist_estep.py)."""
    L = lib()
    if not hasattr(L, "_partial_bound"):
        P = ctypes.c_void_p
        L.oracle_estep_partial.argtypes = [P, P, P, ctypes.c_uint64, P, P, P, ctypes.c_uint64,
                                           ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                           ctypes.c_uint64, P, P, P]
        L._partial_bound = True
    sb, so = to_csr(sentences)
    pb, po = to_csr(pieces)
    fr = np.ascontiguousarray(freqs, dtype=np.int64)
    sc = np.ascontiguousarray(scores, dtype=np.float32)
    L.oracle_estep_partial(_ptr(sb), _ptr(so), _ptr(fr), len(sentences), _ptr(pb), _ptr(po), _ptr(sc),
                           len(pieces), int(all_freq), mode, T, index_base, index_stride, _ptr(acc),
                           _ptr(acc_obj), _ptr(ntok_acc))


def _bind_trainer(L):
    if getattr(L, "_trainer_bound", False):
        return
    P = ctypes.c_void_p
    L.oracle_trainer_create.restype = P
    L.oracle_trainer_create.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, P, P,
                                        ctypes.c_uint64]
    L.oracle_trainer_free.argtypes = [P]
    L.oracle_trainer_sentences.restype = ctypes.c_uint64
    L.oracle_trainer_sentences.argtypes = [P, P, P, P]
    L.oracle_trainer_sentence_bytes.restype = ctypes.c_uint64
    L.oracle_trainer_sentence_bytes.argtypes = [P]
    L.oracle_trainer_seeds.restype = ctypes.c_uint64
    L.oracle_trainer_seeds.argtypes = [P, P, P, P, P]
    L.oracle_trainer_train.restype = ctypes.c_int64
    L.oracle_trainer_train.argtypes = [P, P, P, P, P, P]
    L.oracle_trainer_log.restype = ctypes.c_uint64
    L.oracle_trainer_log.argtypes = [P, P, ctypes.c_uint64]
    L._trainer_bound = True


class OracleTrainer:
    """unigram::Trainer restatement (oracle/spm_oracle_train.inc).  args:
    "--key=value ..." as SentencePieceTrainer::Train(args); charsmap: the
    precompiled charsmap blob of the normalization rule (b"" = identity);
    lines: input lines as ReadLine returns them."""

    def __init__(self, args, lines, charsmap=b""):
        self.L = lib()
        _bind_trainer(self.L)
        buf, off = to_csr(list(lines))
        self.h = self.L.oracle_trainer_create(args.encode(), bytes(charsmap), len(charsmap),
                                              _ptr(buf), _ptr(off), len(lines))
        if not self.h:
            raise ValueError("oracle trainer: bad spec or LoadSentences failed")

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_trainer_free(self.h)
            self.h = None

    def sentences(self):
        n = self.L.oracle_trainer_sentences(self.h, None, None, None)
        nb = self.L.oracle_trainer_sentence_bytes(self.h)
        b = np.zeros(max(nb, 1), dtype=np.uint8)
        o = np.zeros(n + 1, dtype=np.uint64)
        f = np.zeros(max(n, 1), dtype=np.int64)
        self.L.oracle_trainer_sentences(self.h, _ptr(b), _ptr(o), _ptr(f))
        return [b[int(o[i]):int(o[i + 1])].tobytes() for i in range(n)], f[:n].copy()

    def seeds(self):
        nb = np.zeros(1, dtype=np.uint64)
        n = self.L.oracle_trainer_seeds(self.h, None, None, None, _ptr(nb))
        b = np.zeros(max(int(nb[0]), 1), dtype=np.uint8)
        o = np.zeros(n + 1, dtype=np.uint64)
        s = np.zeros(max(n, 1), dtype=np.float32)
        self.L.oracle_trainer_seeds(self.h, _ptr(b), _ptr(o), _ptr(s), None)
        return [b[int(o[i]):int(o[i + 1])].tobytes() for i in range(n)], s[:n].copy()

    def train(self):
        """Runs Train(); returns (pieces, scores float32, types int32) of the
        serialized model (meta pieces included, in id order)."""
        nb = np.zeros(1, dtype=np.uint64)
        n = self.L.oracle_trainer_train(self.h, None, None, None, None, _ptr(nb))
        if n < 0:
            raise RuntimeError("oracle trainer: Train failed")
        b = np.zeros(max(int(nb[0]), 1), dtype=np.uint8)
        o = np.zeros(n + 1, dtype=np.uint64)
        s = np.zeros(max(n, 1), dtype=np.float32)
        t = np.zeros(max(n, 1), dtype=np.int32)
        self.L.oracle_trainer_train(self.h, _ptr(b), _ptr(o), _ptr(s), _ptr(t), None)
        return [b[int(o[i]):int(o[i + 1])].tobytes() for i in range(n)], s[:n].copy(), t[:n].copy()

    def em_log(self):
        n = self.L.oracle_trainer_log(self.h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        self.L.oracle_trainer_log(self.h, buf, n)
        return buf.raw[:n].decode().splitlines()
