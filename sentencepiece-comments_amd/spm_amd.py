"""Python binding of the C-ABI (include/spm_hip.h) via ctypes.

Thin plumbing used by tests/, bench.py and __graft_entry__.py.  The product
is lib/libspm_hip.so; this module never falls back to anything else: if the
library is missing or a call fails, it raises.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SPM_AMD_LIB: another in-tree build of the same library (A/B of kernel
# variants built into a scratch directory, tools/).
LIB_PATH = os.environ.get("SPM_AMD_LIB") or os.path.join(HERE, "lib", "libspm_hip.so")

SPM_OK = 0
SPM_UNIGRAM, SPM_BPE = 1, 2
SPM_ESTEP_FAST, SPM_ESTEP_PARITY = 0, 1
SPM_ESTEP_DEFER_FOLD = 0x100  # include/spm_hip.h

# Every symbol include/spm_hip.h declares.
EXPORTED = [
    "spm_hip_model_load", "spm_hip_model_load_host_only", "spm_hip_model_free", "spm_hip_model_get_info",
    "spm_hip_encode_batch", "spm_hip_encode_batch_host", "spm_hip_normalize_batch",
    "spm_hip_model_set_force_general", "spm_hip_model_set_timing", "spm_hip_model_last_stats",
    "spm_hip_pieces_create", "spm_hip_pieces_free", "spm_hip_pieces_set_scores", "spm_hip_estep", "spm_hip_estep_accumulate",
    "spm_hip_estep_finalize", "spm_hip_estep_sync", "spm_hip_pieces_set_forward", "spm_hip_pieces_last_error", "spm_hip_last_error",
    "spm_hip_model_from_pieces", "spm_hip_seed_mine", "spm_hip_seeds_size", "spm_hip_seeds_bytes",
    "spm_hip_seeds_offsets", "spm_hip_seeds_scores", "spm_hip_seeds_stats", "spm_hip_seeds_free",
    "spm_hip_seed_last_error", "spm_hip_normalize_batch_device", "spm_hip_seed_mine_device",
    "spm_hip_finalize_ids", "spm_hip_model_trie_stats", "spm_hip_estep_shard_plan",
    "spm_hip_normalize_batch_device_align", "spm_hip_encode_spt", "spm_hip_prune_nbest",
    "spm_hip_bpe_pair_census", "spm_hip_bpe_census_free", "spm_hip_bpe_census_last_error",
    "spm_hip_bpe_census_view", "spm_hip_bpe_refresh_create", "spm_hip_bpe_refresh_run",
    "spm_hip_bpe_refresh_stats", "spm_hip_bpe_refresh_free", "spm_hip_encode_batch_async", "spm_hip_normalize_batch_device_async",
    "spm_hip_finalize_ids_async", "spm_hip_model_drain_kernel_times", "spm_hip_model_set_debug_corrupt_bp",
    "spm_hip_model_set_coop_min_nb",
    "spm_hip_model_set_coop_slab",
    "spm_hip_model_release_stream", "spm_hip_abi_version", "spm_hip_seeds_stage_times",
    "spm_hip_estep_record_stats", "spm_hip_estep_bucket_owner", "spm_hip_pieces_set_timing",
    "spm_hip_estep_kernel_times", "spm_hip_device_bytes", "spm_hip_device_peak_reset",
    "spm_hip_encode_raw_small_host",
]

ABI_VERSION = 3  # SPM_HIP_ABI_VERSION of include/spm_hip.h (struct layouts below)


def device_bytes():
    """spm_hip_device_bytes: (live, peak) device bytes this library holds in
    the process (peak since the last device_peak_reset)."""
    live, peak = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _check(lib().spm_hip_device_bytes(ctypes.byref(live), ctypes.byref(peak)))
    return live.value, peak.value


def device_peak_reset():
    lib().spm_hip_device_peak_reset()


def estep_shard_plan(n, mode, num_threads, world, rank):
    """spm_hip_estep_shard_plan: rank's E-step segments [(index_base,
    index_stride, count)] (host only; csrc/shard_plan.h)."""
    L = lib()
    cnt = ctypes.c_uint64(0)
    _check(L.spm_hip_estep_shard_plan(n, mode, num_threads, world, rank, None, 0, ctypes.byref(cnt)))
    buf = np.zeros(3 * max(cnt.value, 1), dtype=np.uint64)
    _check(L.spm_hip_estep_shard_plan(n, mode, num_threads, world, rank,
                                      buf.ctypes.data_as(ctypes.c_void_p), cnt.value, ctypes.byref(cnt)))
    return [tuple(int(x) for x in buf[3 * k:3 * k + 3]) for k in range(cnt.value)]


def estep_bucket_owner(bucket, num_threads, world):
    """spm_hip_estep_bucket_owner: the rank holding PARITY bucket `bucket`
    (the row spm_train's reduction gathers from it); -1 if invalid."""
    return int(lib().spm_hip_estep_bucket_owner(bucket, num_threads, world))


class SpmError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("spm_hip error %d: %s" % (code, msg))
        self.code = code


class ModelInfo(ctypes.Structure):
    _fields_ = [("model_type", ctypes.c_int32), ("piece_size", ctypes.c_int32),
                ("unk_id", ctypes.c_int32), ("max_piece_chars", ctypes.c_int32),
                ("trie_results_size", ctypes.c_int32), ("trie_units", ctypes.c_int32),
                ("min_score", ctypes.c_float), ("max_score", ctypes.c_float),
                ("ring_width", ctypes.c_int32), ("fast_variant", ctypes.c_int32)]


class TrieStats(ctypes.Structure):
    _fields_ = [("char_starts", ctypes.c_uint64), ("unit_loads", ctypes.c_uint64),
                ("leaf_loads", ctypes.c_uint64), ("max_depth", ctypes.c_uint64),
                ("units_below", ctypes.c_uint64 * 8), ("lockstep_rounds", ctypes.c_uint64),
                ("decoupled_rounds", ctypes.c_uint64), ("waves", ctypes.c_uint64)]


class SeedOptions(ctypes.Structure):
    _fields_ = [("max_sentencepiece_length", ctypes.c_int32),
                ("split_by_unicode_script", ctypes.c_int32), ("split_by_number", ctypes.c_int32),
                ("split_by_whitespace", ctypes.c_int32),
                ("treat_whitespace_as_suffix", ctypes.c_int32),
                ("seed_sentencepiece_size", ctypes.c_int64)]


class EncodeStats(ctypes.Structure):
    _fields_ = [("sentences", ctypes.c_uint64), ("tokens", ctypes.c_uint64),
                ("general_path", ctypes.c_uint64), ("fast_kernel_ms", ctypes.c_float),
                ("general_kernel_ms", ctypes.c_float), ("coop_rest", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libspm_hip.so not built: run `make -C sentencepiece-comments_amd` "
                              "(or __graft_entry__.build())")
        # torch bundles its own libamdhip64 (SONAME libamdhip64.so.7).  Load it
        # first so libspm_hip.so binds to that same runtime; otherwise two HIP
        # runtimes end up in one process and torch sees no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        P, U64, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.spm_hip_model_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(P)]
        L.spm_hip_model_load_host_only.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(P)]
        L.spm_hip_model_free.argtypes = [P]
        L.spm_hip_model_free.restype = None
        L.spm_hip_model_get_info.argtypes = [P, ctypes.POINTER(ModelInfo)]
        L.spm_hip_encode_batch.argtypes = [P, P, P, U64, P, P, P, P]
        L.spm_hip_encode_batch_async.argtypes = [P, P, P, U64, U64, P, P, P, P, P]
        L.spm_hip_normalize_batch_device_async.argtypes = [P, P, P, U64, P, U64, P, P, P, P]
        L.spm_hip_finalize_ids_async.argtypes = [P, ctypes.c_char_p, P, P, U64, P, U64, P, P, P]
        L.spm_hip_model_drain_kernel_times.argtypes = [P, P, P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        L.spm_hip_model_set_debug_corrupt_bp.argtypes = [P, ctypes.c_int64]
        L.spm_hip_model_set_coop_min_nb.argtypes = [P, ctypes.c_uint32]
        L.spm_hip_model_set_coop_slab.argtypes = [P, ctypes.c_int, ctypes.c_uint32]
        L.spm_hip_model_release_stream.argtypes = [P, P]
        if L.spm_hip_abi_version() != ABI_VERSION:
            raise ImportError("libspm_hip.so ABI version %d, binding expects %d"
                              % (L.spm_hip_abi_version(), ABI_VERSION))
        L.spm_hip_encode_batch_host.argtypes = [P, P, P, U64, P, P, P]
        L.spm_hip_normalize_batch.argtypes = [P, P, P, U64, P, P, I]
        L.spm_hip_model_set_force_general.argtypes = [P, I]
        L.spm_hip_model_set_timing.argtypes = [P, I]
        L.spm_hip_model_last_stats.argtypes = [P, ctypes.POINTER(EncodeStats)]
        L.spm_hip_pieces_create.argtypes = [P, P, P, U64, ctypes.POINTER(P)]
        L.spm_hip_pieces_free.argtypes = [P]
        L.spm_hip_pieces_free.restype = None
        L.spm_hip_pieces_set_scores.argtypes = [P, P, U64]
        L.spm_hip_pieces_set_scores.restype = ctypes.c_int
        L.spm_hip_estep.argtypes = [P, P, P, P, U64, ctypes.c_int64, I, I, P, P, P, P]
        L.spm_hip_estep_accumulate.argtypes = [P, P, P, P, U64, ctypes.c_int64, I, I, U64, U64,
                                               P, P, P, P]
        L.spm_hip_estep_finalize.argtypes = [P, I, I, P, P, P, P, P, P, P]
        L.spm_hip_estep_sync.argtypes = [P, P]
        L.spm_hip_pieces_set_forward.argtypes = [P, I]
        L.spm_hip_estep_record_stats.argtypes = [P, ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.spm_hip_pieces_set_timing.argtypes = [P, I]
        L.spm_hip_estep_kernel_times.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(U64)]
        L.spm_hip_prune_nbest.argtypes = [P, P, P, P, P, P, P, ctypes.c_uint32, P]
        L.spm_hip_estep_shard_plan.argtypes = [U64, I, I, I, I, P, U64, ctypes.POINTER(U64)]
        L.spm_hip_estep_bucket_owner.argtypes = [I, I, I]
        L.spm_hip_normalize_batch_device_align.argtypes = [P, P, P, U64, P, U64, P, P, ctypes.POINTER(U64), P]
        L.spm_hip_encode_spt.argtypes = [P, ctypes.c_char_p, P, P, U64, P, U64, P, P, P, U64, P,
                                         ctypes.POINTER(U64), ctypes.POINTER(U64), P]
        L.spm_hip_pieces_last_error.argtypes = [P]
        L.spm_hip_pieces_last_error.restype = ctypes.c_char_p
        L.spm_hip_last_error.restype = ctypes.c_char_p
        L.spm_hip_normalize_batch_device.argtypes = [P, P, P, U64, P, U64, P, ctypes.POINTER(U64), P]
        L.spm_hip_model_from_pieces.argtypes = [P, P, P, U64, ctypes.POINTER(P)]
        L.spm_hip_finalize_ids.argtypes = [P, ctypes.c_char_p, P, P, U64, P, U64, P, ctypes.POINTER(U64), P]
        L.spm_hip_seed_mine.argtypes = [P, P, U64, P, P, U64, ctypes.POINTER(SeedOptions),
                                        ctypes.POINTER(P)]
        L.spm_hip_seeds_size.argtypes = [P]
        L.spm_hip_seeds_size.restype = U64
        for fn in ("spm_hip_seeds_bytes", "spm_hip_seeds_offsets", "spm_hip_seeds_scores"):
            getattr(L, fn).argtypes = [P]
            getattr(L, fn).restype = P
        L.spm_hip_seeds_stats.argtypes = [P, P, P, P]
        L.spm_hip_seeds_free.argtypes = [P]
        L.spm_hip_seeds_free.restype = None
        L.spm_hip_seed_last_error.restype = ctypes.c_char_p
        L.spm_hip_model_trie_stats.argtypes = [P, P, P, U64, I, ctypes.POINTER(TrieStats)]
        L.spm_hip_device_bytes.argtypes = [ctypes.POINTER(U64), ctypes.POINTER(U64)]
        L.spm_hip_encode_raw_small_host.argtypes = [P, P, P, U64, P, U64, P]
        L.spm_hip_device_peak_reset.restype = None
        _lib = L
    return _lib


def _check(rc):
    if rc != SPM_OK:
        raise SpmError(rc, lib().spm_hip_last_error().decode(errors="replace"))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def to_csr(items):
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    buf = np.frombuffer(b"".join(items), dtype=np.uint8).copy()
    if buf.size == 0:
        buf = np.zeros(1, dtype=np.uint8)
    return buf, off


class DeviceModel:
    """A model resident on the current HIP device (spm_hip_model handle)."""

    def __init__(self, model_bytes, host_only=False):
        self._L = lib()
        h = ctypes.c_void_p()
        b = bytes(model_bytes)
        fn = self._L.spm_hip_model_load_host_only if host_only else self._L.spm_hip_model_load
        _check(fn(b, len(b), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._L.spm_hip_model_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def info(self):
        inf = ModelInfo()
        _check(self._L.spm_hip_model_get_info(self.h, ctypes.byref(inf)))
        return inf

    def trie_stats(self, buf, off, threads=0):
        """Diagnostic: trie unit/leaf loads of unigram Encode over a host CSR batch."""
        ts = TrieStats()
        _check(self._L.spm_hip_model_trie_stats(self.h, _p(buf), _p(off), len(off) - 1, threads,
                                                 ctypes.byref(ts)))
        return ts

    def stats(self):
        st = EncodeStats()
        _check(self._L.spm_hip_model_last_stats(self.h, ctypes.byref(st)))
        return st

    def set_timing(self, on):
        _check(self._L.spm_hip_model_set_timing(self.h, 1 if on else 0))

    def set_force_general(self, on):
        _check(self._L.spm_hip_model_set_force_general(self.h, 1 if on else 0))

    def set_debug_corrupt_bp(self, sentence):
        """Debug knob: zero this sentence's EOS back-pointer in the fast kernel (-1: off)."""
        _check(self._L.spm_hip_model_set_debug_corrupt_bp(self.h, int(sentence)))

    def set_coop_min_nb(self, min_nb):
        """Wide / char kernel models: sentences of >= min_nb bytes take the
        wave-cooperative kernel (0: none)."""
        _check(self._L.spm_hip_model_set_coop_min_nb(self.h, int(min_nb)))

    def set_coop_slab(self, mode, slab_chars=0):
        """Cooperative-kernel scratch rows: 0 auto, 1 per-wave slabs of
        slab_chars chars (0: default), 2 by byte offset."""
        _check(self._L.spm_hip_model_set_coop_slab(self.h, int(mode), int(slab_chars)))

    def release_stream(self, stream):
        _check(self._L.spm_hip_model_release_stream(self.h, ctypes.c_void_p(stream) if stream else None))

    def drain_kernel_times(self, stream=None):
        """Fast-kernel durations (ms) of the encode calls on `stream` since the last drain."""
        buf = np.zeros(64, dtype=np.float32)
        cnt = ctypes.c_uint32()
        _check(self._L.spm_hip_model_drain_kernel_times(self.h, ctypes.c_void_p(stream) if stream else None,
                                                         _p(buf), 64, ctypes.byref(cnt)))
        return buf[:cnt.value].tolist()

    def normalize_csr(self, buf, off, threads=0):
        n = len(off) - 1
        out = np.zeros(int(off[-1]) * 3 + 3 * n + 16, dtype=np.uint8)
        oo = np.zeros(n + 1, dtype=np.uint64)
        _check(self._L.spm_hip_normalize_batch(self.h, _p(buf), _p(off), n, _p(out), _p(oo), threads))
        return out[:int(oo[-1])].copy() if int(oo[-1]) else np.zeros(1, np.uint8), oo

    def normalize(self, lines, threads=0):
        buf, off = to_csr(lines)
        out, oo = self.normalize_csr(buf, off, threads)
        b = out.tobytes()
        return [b[int(oo[i]):int(oo[i + 1])] for i in range(len(lines))]

    def normalize_device(self, lines):
        """Normalizer on the device (spm_hip_normalize_batch_device); host
        lists in and out, torch for the device buffers."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        buf, off = to_csr(lines)
        n = len(lines)
        d_in = torch.from_numpy(buf).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_oo = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        cap = int(off[-1]) * 3 + 3 * n + 16
        d_out = torch.zeros(max(cap, 1), dtype=torch.uint8, device=dev)
        tot = ctypes.c_uint64()
        s = torch.cuda.current_stream(dev).cuda_stream
        rc = self._L.spm_hip_normalize_batch_device(self.h, d_in.data_ptr(), d_off.data_ptr(), n,
                                                    d_out.data_ptr(), cap, d_oo.data_ptr(),
                                                    ctypes.byref(tot), s)
        if rc == 8:  # RESOURCE_EXHAUSTED: grow and retry once
            cap = tot.value
            d_out = torch.zeros(max(cap, 1), dtype=torch.uint8, device=dev)
            rc = self._L.spm_hip_normalize_batch_device(self.h, d_in.data_ptr(), d_off.data_ptr(), n,
                                                        d_out.data_ptr(), cap, d_oo.data_ptr(),
                                                        ctypes.byref(tot), s)
        _check(rc)
        torch.cuda.synchronize(dev)
        b = d_out[:tot.value].cpu().numpy().tobytes()
        oo = d_oo.cpu().numpy()
        return [b[int(oo[i]):int(oo[i + 1])] for i in range(n)]

    def normalize_align_device(self, lines):
        """spm_hip_normalize_batch_device_align: [(normalized bytes,
        norm_to_orig list of len + 1)] per line."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        buf, off = to_csr(lines)
        n = len(lines)
        d_in = torch.from_numpy(buf).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_oo = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        cap = int(off[-1]) * 3 + 3 * n + 16
        d_out = torch.zeros(cap, dtype=torch.uint8, device=dev)
        d_a = torch.zeros(cap + n, dtype=torch.int32, device=dev)
        tot = ctypes.c_uint64()
        s = torch.cuda.current_stream(dev).cuda_stream
        _check(self._L.spm_hip_normalize_batch_device_align(self.h, d_in.data_ptr(), d_off.data_ptr(), n,
                                                            d_out.data_ptr(), cap, d_oo.data_ptr(),
                                                            d_a.data_ptr(), ctypes.byref(tot), s))
        torch.cuda.synchronize(dev)
        b = d_out[:tot.value].cpu().numpy().tobytes()
        oo = d_oo.cpu().numpy()
        a = d_a.cpu().numpy().view(np.uint32)
        return [(b[int(oo[i]):int(oo[i + 1])], a[int(oo[i]) + i:int(oo[i + 1]) + i + 1].tolist())
                for i in range(n)]

    def encode_spt_device(self, lines, extra_options=""):
        """spm_hip_encode_spt: SentencePieceProcessor::Encode(SentencePieceText)
        per raw line, all on the device.  Returns per line
        [(id, piece bytes, surface bytes, begin, end)], the piece string taken
        from the normalized bytes (None for the bos/eos extras, whose piece is
        IdToPiece(id))."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        buf, off = to_csr(lines)
        n = len(lines)
        s = torch.cuda.current_stream(dev).cuda_stream
        d_in = torch.from_numpy(buf).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        cap = int(off[-1]) * 3 + 3 * n + 16
        d_norm = torch.empty(cap, dtype=torch.uint8, device=dev)
        d_noff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_a = torch.empty(cap + n, dtype=torch.int32, device=dev)
        pcap = cap + 2 * 32 * n
        d_p = torch.empty(pcap * 5, dtype=torch.int32, device=dev)
        d_po = torch.empty(n + 1, dtype=torch.int64, device=dev)
        tn, tp = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._L.spm_hip_encode_spt(self.h, extra_options.encode(), d_in.data_ptr(), d_off.data_ptr(), n,
                                          d_norm.data_ptr(), cap, d_noff.data_ptr(), d_a.data_ptr(),
                                          d_p.data_ptr(), pcap, d_po.data_ptr(), ctypes.byref(tn),
                                          ctypes.byref(tp), s))
        torch.cuda.synchronize(dev)
        nb = d_norm[:tn.value].cpu().numpy().tobytes()
        no = d_noff.cpu().numpy()
        p = d_p[:5 * tp.value].cpu().numpy().reshape(-1, 5)
        po = d_po.cpu().numpy()
        out = []
        for i in range(n):
            norm = nb[int(no[i]):int(no[i + 1])]
            row = []
            for k in range(int(po[i]), int(po[i + 1])):
                pid, b, e, nb0, ne0 = (int(x) for x in p[k].view(np.int32)[:1].tolist() +
                                       p[k].view(np.uint32)[1:].tolist())
                piece = norm[nb0:ne0] if ne0 > nb0 else None
                row.append((pid, piece, lines[i][b:e], b, e))
            out.append(row)
        return out

    def encode_csr_host(self, buf, off, with_lens=False):
        """Host CSR in → (ids int32, [piece_len uint32], tok_off uint64[n+1])."""
        n = len(off) - 1
        cap = max(int(off[-1]), 1)
        ids = np.zeros(cap, dtype=np.int32)
        lens = np.zeros(cap, dtype=np.uint32) if with_lens else None
        to = np.zeros(n + 1, dtype=np.uint64)
        _check(self._L.spm_hip_encode_batch_host(self.h, _p(buf), _p(off), n, _p(ids),
                                                 _p(lens) if with_lens else None, _p(to)))
        k = int(to[-1])
        if with_lens:
            return ids[:k], lens[:k], to
        return ids[:k], to

    def encode_normalized(self, sentences):
        buf, off = to_csr(sentences)
        ids, to = self.encode_csr_host(buf, off)
        return [ids[int(to[i]):int(to[i + 1])].tolist() for i in range(len(sentences))]

    def encode_device(self, d_bytes, d_off, n, d_ids, d_tok, d_len=None, stream=None):
        """Device pointers (ints, e.g. torch tensor .data_ptr()); async on stream."""
        _check(self._L.spm_hip_encode_batch(self.h, ctypes.c_void_p(d_bytes), ctypes.c_void_p(d_off),
                                            n, ctypes.c_void_p(d_ids),
                                            ctypes.c_void_p(d_len) if d_len else None,
                                            ctypes.c_void_p(d_tok),
                                            ctypes.c_void_p(stream) if stream else None))

    def encode_device_async(self, d_bytes, d_off, n, capacity, d_ids, d_tok, d_status, d_len=None, stream=None):
        """spm_hip_encode_batch_async: pure stream call (no host synchronization);
        failures land in the device status word d_status."""
        V = ctypes.c_void_p
        _check(self._L.spm_hip_encode_batch_async(self.h, V(d_bytes), V(d_off), n, capacity, V(d_ids),
                                                  V(d_len) if d_len else None, V(d_tok), V(d_status),
                                                  V(stream) if stream else None))

    def normalize_device_async(self, d_in, d_in_off, n, d_out, out_capacity, d_out_off, d_status, d_n2o=None,
                               stream=None):
        V = ctypes.c_void_p
        _check(self._L.spm_hip_normalize_batch_device_async(self.h, V(d_in), V(d_in_off), n, V(d_out),
                                                            out_capacity, V(d_out_off),
                                                            V(d_n2o) if d_n2o else None, V(d_status),
                                                            V(stream) if stream else None))

    def finalize_ids_device_async(self, extra_options, d_ids, d_tok, n, d_out, out_capacity, d_out_off, d_status,
                                  stream=None):
        V = ctypes.c_void_p
        _check(self._L.spm_hip_finalize_ids_async(self.h, extra_options.encode(), V(d_ids), V(d_tok), n, V(d_out),
                                                  out_capacity, V(d_out_off), V(d_status),
                                                  V(stream) if stream else None))

    def encode_lines_device_async(self, lines, extra_options=""):
        """encode_lines_device through the pure stream calls (normalize →
        encode → id epilogue, one status word, one synchronization at the
        end).  Returns (per-line ids, status code)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        buf, off = to_csr(lines)
        n = len(lines)
        s = torch.cuda.current_stream(dev).cuda_stream
        d_in = torch.from_numpy(buf).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        cap = int(off[-1]) * 3 + 3 * n + 16
        d_norm = torch.empty(cap, dtype=torch.uint8, device=dev)
        d_noff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
        d_tok = torch.empty(n + 1, dtype=torch.int64, device=dev)
        n_extra = sum(1 for o in extra_options.split(":") if o in ("bos", "eos"))
        ocap = cap + n * n_extra
        d_out = torch.empty(max(ocap, 1), dtype=torch.int32, device=dev)
        d_ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_st = torch.zeros(1, dtype=torch.int32, device=dev)
        self.normalize_device_async(d_in.data_ptr(), d_off.data_ptr(), n, d_norm.data_ptr(), cap, d_noff.data_ptr(),
                                    d_st.data_ptr(), stream=s)
        self.encode_device_async(d_norm.data_ptr(), d_noff.data_ptr(), n, cap, d_ids.data_ptr(), d_tok.data_ptr(),
                                 d_st.data_ptr(), stream=s)
        self.finalize_ids_device_async(extra_options, d_ids.data_ptr(), d_tok.data_ptr(), n, d_out.data_ptr(), ocap,
                                       d_ooff.data_ptr(), d_st.data_ptr(), stream=s)
        torch.cuda.synchronize(dev)
        code = int(d_st.item())
        if code:
            return None, code
        oo = d_ooff.cpu().numpy()
        out = d_out[:int(oo[-1])].cpu().numpy()
        return [out[int(oo[i]):int(oo[i + 1])].tolist() for i in range(n)], 0

    def finalize_ids_device(self, extra_options, d_ids, d_tok, n, d_out, out_capacity, d_out_off,
                            stream=None):
        """spm_hip_finalize_ids (unk-run merge + extra options) on device
        pointers; returns the output id count."""
        tot = ctypes.c_uint64()
        _check(self._L.spm_hip_finalize_ids(self.h, extra_options.encode(), ctypes.c_void_p(d_ids),
                                            ctypes.c_void_p(d_tok), n, ctypes.c_void_p(d_out),
                                            out_capacity, ctypes.c_void_p(d_out_off), ctypes.byref(tot),
                                            ctypes.c_void_p(stream) if stream else None))
        return tot.value

    def encode_raw_small(self, lines):
        """spm_hip_encode_raw_small_host: raw lines -> final ids (Encode(line,
        &ids), no extra options) in one launch; None when the fused path does
        not take the call (SPM_UNIMPLEMENTED)."""
        buf, off = to_csr(lines)
        n = len(lines)
        cap = int(off[-1]) * 4 + 8 * n + 64
        ids = np.zeros(max(cap, 1), dtype=np.int32)
        to = np.zeros(n + 1, dtype=np.uint64)
        rc = self._L.spm_hip_encode_raw_small_host(self.h, _p(buf), _p(off), n, _p(ids), cap, _p(to))
        if rc == 12:  # SPM_UNIMPLEMENTED
            return None
        _check(rc)
        return [ids[int(to[i]):int(to[i + 1])].tolist() for i in range(n)]

    def encode_lines_device(self, lines, extra_options=""):
        """Raw lines → final ids, all on the device: Normalize
        (spm_hip_normalize_batch_device) + Encode (spm_hip_encode_batch) +
        id epilogue (spm_hip_finalize_ids) — SentencePieceProcessor::Encode(ids)
        per line.  Host lists in and out, torch for the device buffers."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        buf, off = to_csr(lines)
        n = len(lines)
        s = torch.cuda.current_stream(dev).cuda_stream
        d_in = torch.from_numpy(buf).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        cap = int(off[-1]) * 3 + 3 * n + 16
        d_norm = torch.empty(cap, dtype=torch.uint8, device=dev)
        d_noff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        tot = ctypes.c_uint64()
        _check(self._L.spm_hip_normalize_batch_device(self.h, d_in.data_ptr(), d_off.data_ptr(), n,
                                                      d_norm.data_ptr(), cap, d_noff.data_ptr(),
                                                      ctypes.byref(tot), s))
        d_ids = torch.empty(max(tot.value, 1), dtype=torch.int32, device=dev)
        d_tok = torch.empty(n + 1, dtype=torch.int64, device=dev)
        self.encode_device(d_norm.data_ptr(), d_noff.data_ptr(), n, d_ids.data_ptr(), d_tok.data_ptr(),
                           stream=s)
        n_extra = sum(1 for o in extra_options.split(":") if o in ("bos", "eos"))
        ocap = tot.value + n * n_extra
        d_out = torch.empty(max(ocap, 1), dtype=torch.int32, device=dev)
        d_ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        k = self.finalize_ids_device(extra_options, d_ids.data_ptr(), d_tok.data_ptr(), n, d_out.data_ptr(),
                                     ocap, d_ooff.data_ptr(), stream=s)
        torch.cuda.synchronize(dev)
        out = d_out[:k].cpu().numpy()
        oo = d_ooff.cpu().numpy()
        return [out[int(oo[i]):int(oo[i + 1])].tolist() for i in range(n)]


class DevicePieces:
    """TrainerModel piece list resident on the device (spm_hip_pieces)."""

    def __init__(self, pieces, scores):
        self._L = lib()
        buf, off = to_csr([p if isinstance(p, bytes) else p.encode() for p in pieces])
        sc = np.ascontiguousarray(scores, dtype=np.float32)
        h = ctypes.c_void_p()
        rc = self._L.spm_hip_pieces_create(_p(buf), _p(off), _p(sc), len(pieces), ctypes.byref(h))
        if rc != SPM_OK:
            raise SpmError(rc, "spm_hip_pieces_create failed")
        self.h = h
        self.V = len(pieces)

    def close(self):
        if getattr(self, "h", None):
            self._L.spm_hip_pieces_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != SPM_OK:
            raise SpmError(rc, self._L.spm_hip_pieces_last_error(self.h).decode(errors="replace"))

    def estep_device(self, d_bytes, d_off, d_freq, n, all_freq, mode, threads, d_expected, d_obj,
                     d_ntok, stream=None):
        V = ctypes.c_void_p
        self._check(self._L.spm_hip_estep(self.h, V(d_bytes), V(d_off), V(d_freq), n, all_freq, mode,
                                          threads, V(d_expected), V(d_obj), V(d_ntok),
                                          V(stream) if stream else None))

    def accumulate_device(self, d_bytes, d_off, d_freq, n, all_freq, mode, threads, index_base,
                          index_stride, d_acc, d_acc_obj, d_ntok_acc, stream=None, defer=False):
        """defer: SPM_ESTEP_DEFER_FOLD (the accumulators are complete on the
        stream only after sync_device or finalize_device)."""
        V = ctypes.c_void_p
        self._check(self._L.spm_hip_estep_accumulate(
            self.h, V(d_bytes), V(d_off), V(d_freq), n, all_freq, mode | (SPM_ESTEP_DEFER_FOLD if defer else 0),
            threads, index_base, index_stride, V(d_acc), V(d_acc_obj), V(d_ntok_acc),
            V(stream) if stream else None))

    def set_scores(self, scores):
        """spm_hip_pieces_set_scores: new scores for the same piece list."""
        sc = np.ascontiguousarray(scores, dtype=np.float32)
        if len(sc) != self.V:
            raise ValueError("set_scores needs one score per piece")
        self._check(self._L.spm_hip_pieces_set_scores(self.h, _p(sc), self.V))

    def set_forward(self, mode):
        """spm_hip_pieces_set_forward: 0 auto, 1 byte-kernel E-step mode, 2 estep_forward_kernel."""
        self._check(self._L.spm_hip_pieces_set_forward(self.h, mode))

    def record_stats(self):
        """spm_hip_estep_record_stats: (PARITY records written, records kept
        after the no-op drop) since the piece set was created."""
        w, k = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self._L.spm_hip_estep_record_stats(self.h, ctypes.byref(w), ctypes.byref(k)))
        return int(w.value), int(k.value)

    def set_timing(self, on):
        """spm_hip_pieces_set_timing: HIP events around each chunk's forward and backward pass."""
        self._check(self._L.spm_hip_pieces_set_timing(self.h, 1 if on else 0))

    def kernel_times(self):
        """spm_hip_estep_kernel_times: (forward ms, backward ms, chunks) since the last call."""
        f, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        self._check(self._L.spm_hip_estep_kernel_times(self.h, ctypes.byref(f), ctypes.byref(b), ctypes.byref(c)))
        return float(f.value), float(b.value), int(c.value)

    def sync_device(self, stream=None):
        """spm_hip_estep_sync: `stream` waits for every deferred fold."""
        self._check(self._L.spm_hip_estep_sync(self.h, ctypes.c_void_p(stream) if stream else None))

    def finalize_device(self, mode, threads, d_acc, d_acc_obj, d_ntok_acc, d_expected, d_obj, d_ntok,
                        stream=None):
        V = ctypes.c_void_p
        self._check(self._L.spm_hip_estep_finalize(self.h, mode, threads, V(d_acc), V(d_acc_obj),
                                                   V(d_ntok_acc), V(d_expected), V(d_obj), V(d_ntok),
                                                   V(stream) if stream else None))

    def estep(self, sentences, freqs, mode=SPM_ESTEP_FAST, threads=1):
        """Host convenience (uses torch for device buffers)."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        buf, off = to_csr(sentences)
        d_b = torch.from_numpy(buf).to(dev)
        d_o = torch.from_numpy(off.view(np.int64)).to(dev)
        fr = np.ascontiguousarray(freqs, dtype=np.int64)
        d_f = torch.from_numpy(fr).to(dev)
        d_e = torch.zeros(self.V, dtype=torch.float32, device=dev)
        d_obj = torch.zeros(1, dtype=torch.float32, device=dev)
        d_nt = torch.zeros(1, dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        self.estep_device(d_b.data_ptr(), d_o.data_ptr(), d_f.data_ptr(), len(sentences),
                          int(fr.sum()), mode, threads, d_e.data_ptr(), d_obj.data_ptr(),
                          d_nt.data_ptr(), s)
        torch.cuda.synchronize(dev)
        return d_e.cpu().numpy(), float(d_obj.item()), int(d_nt.item())


def seed_mine(sentences, chars, char_freq, max_sentencepiece_length=16, split_by_unicode_script=True,
              split_by_number=True, split_by_whitespace=True, treat_whitespace_as_suffix=False,
              seed_sentencepiece_size=1000000):
    """spm_hip_seed_mine (MakeSeedSentencePieces on the device).  sentences:
    list[bytes] after LoadSentences; chars/char_freq: required chars (code
    points) and their freq-weighted counts.  Returns (pieces list[bytes],
    scores float32, stats dict)."""
    L = lib()
    buf, off = to_csr(list(sentences))
    ch = np.ascontiguousarray(chars, dtype=np.uint32)
    fr = np.ascontiguousarray(char_freq, dtype=np.int64)
    o = SeedOptions(max_sentencepiece_length, int(split_by_unicode_script), int(split_by_number),
                    int(split_by_whitespace), int(treat_whitespace_as_suffix), seed_sentencepiece_size)
    h = ctypes.c_void_p()
    rc = L.spm_hip_seed_mine(_p(buf), _p(off), len(sentences), _p(ch), _p(fr), len(ch),
                             ctypes.byref(o), ctypes.byref(h))
    if rc != SPM_OK:
        raise SpmError(rc, L.spm_hip_seed_last_error().decode(errors="replace"))
    try:
        k = L.spm_hip_seeds_size(h)
        so = np.ctypeslib.as_array(ctypes.cast(L.spm_hip_seeds_offsets(h), ctypes.POINTER(ctypes.c_uint64)),
                                   shape=(k + 1,)).copy()
        nb = int(so[-1])
        b = ctypes.string_at(L.spm_hip_seeds_bytes(h), nb) if nb else b""
        sc = np.ctypeslib.as_array(ctypes.cast(L.spm_hip_seeds_scores(h), ctypes.POINTER(ctypes.c_float)),
                                   shape=(k,)).copy() if k else np.zeros(0, np.float32)
        nc, cand, ms = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_float()
        L.spm_hip_seeds_stats(h, ctypes.byref(nc), ctypes.byref(cand), ctypes.byref(ms))
        pieces = [b[int(so[i]):int(so[i + 1])] for i in range(k)]
        return pieces, sc, {"num_chars": nc.value, "candidates": cand.value, "device_ms": ms.value}
    finally:
        L.spm_hip_seeds_free(h)
