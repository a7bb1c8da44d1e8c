"""Sharded unigram E-step across GPUs (one process per GPU, RCCL over xGMI).

The reference runs RunEStep on T threads of one host and sums the T per-thread
float vectors in thread order (unigram_model_trainer.cc:237-287).  Here each
rank accumulates its shard on its GPU (spm_hip_estep_accumulate) and the
accumulators are summed with ONE all-reduce per EM sub-iteration:

  FAST   : contiguous sentence shards; acc = fp64[V] (+ obj fp64, ntok int64);
           SUM all-reduce, then rounding to float once (spm_hip_estep_finalize).
  PARITY : bucket b = global index mod T (the reference's thread of that
           sentence); rank r owns the buckets b with b % W == r and accumulates
           each bucket's sentences in ascending order into acc = float[T][V].
           Other ranks hold exact zeros in those rows, so the SUM all-reduce
           is exact and finalize sums the buckets in order 0..T-1, bit-equal
           to the reference at num_threads = T.

The accumulate / finalize callables are injected so the same driver runs on
the GPU (DeviceEStep) and, in the CPU tests, on the oracle under gloo.
"""
import numpy as np

FAST, PARITY = 0, 1


def contiguous_shard(n, world, rank):
    return n * rank // world, n * (rank + 1) // world


def owned_buckets(T, world, rank):
    return [b for b in range(T) if b % world == rank]


def plan_chunks(sentences, freqs, mode, T, world, rank):
    """Host corpus → this rank's chunks: list of (sentences, freqs, index_base, index_stride)."""
    n = len(sentences)
    if mode == FAST:
        lo, hi = contiguous_shard(n, world, rank)
        return [(sentences[lo:hi], np.asarray(freqs[lo:hi]), lo, 1)] if hi > lo else []
    chunks = []
    for b in owned_buckets(T, world, rank):
        idx = range(b, n, T)
        if len(idx) == 0:
            continue
        chunks.append(([sentences[i] for i in idx], np.asarray([freqs[i] for i in idx]), b, T))
    return chunks


def accumulator_shapes(mode, T, V):
    """(acc, acc_obj, ntok_acc) shapes and numpy dtypes."""
    if mode == FAST:
        return ((V,), np.float64), ((1,), np.float64), ((1,), np.int64)
    return ((T * V,), np.float32), ((T,), np.float32), ((T,), np.int64)


def finalize_host(mode, T, V, acc, acc_obj, ntok_acc):
    """Host mirror of estep_finalize_kernel (used by CPU tests)."""
    if mode == FAST:
        return acc.astype(np.float32), float(np.float32(acc_obj[0])), int(ntok_acc[0])
    e = acc[:V].copy()
    o = np.float32(acc_obj[0])
    for t in range(1, T):
        e = (e + acc[t * V:(t + 1) * V]).astype(np.float32)
        o = np.float32(o + acc_obj[t])
    return e, float(o), int(ntok_acc.sum())


def run_sharded(chunks, mode, T, V, accumulate, finalize, make_zeros, all_reduce=None):
    """Generic driver.  accumulate(chunk, acc, acc_obj, ntok_acc); all_reduce(x)
    sums a buffer in place across ranks (None for a single process)."""
    (sa, da), (so, do), (sn, dn) = accumulator_shapes(mode, T, V)
    acc, acc_obj, ntok_acc = make_zeros(sa, da), make_zeros(so, do), make_zeros(sn, dn)
    for c in chunks:
        accumulate(c, acc, acc_obj, ntok_acc)
    if all_reduce is not None:
        all_reduce(acc)
        all_reduce(acc_obj)
        all_reduce(ntok_acc)
    return finalize(acc, acc_obj, ntok_acc)


class DeviceEStep:
    """GPU accumulate/finalize over torch device tensors (RCCL all-reduce)."""

    def __init__(self, device_pieces, mode, T, device, all_sentence_freq):
        import torch
        self.torch = torch
        self.dp = device_pieces
        self.mode, self.T, self.dev = mode, T, device
        self.all_freq = int(all_sentence_freq)

    def upload(self, sentences, freqs, index_base, index_stride):
        import spm_amd
        buf, off = spm_amd.to_csr(sentences)
        t = self.torch
        return {"b": t.from_numpy(buf).to(self.dev), "o": t.from_numpy(off.view(np.int64)).to(self.dev),
                "f": t.from_numpy(np.ascontiguousarray(freqs, dtype=np.int64)).to(self.dev),
                "n": len(sentences), "base": index_base, "stride": index_stride}

    def make_zeros(self, shape, dtype):
        tdt = {np.float64: self.torch.float64, np.float32: self.torch.float32,
               np.int64: self.torch.int64}[dtype]
        return self.torch.zeros(shape, dtype=tdt, device=self.dev)

    def accumulate(self, c, acc, acc_obj, ntok_acc):
        s = self.torch.cuda.current_stream(self.dev).cuda_stream
        self.dp.accumulate_device(c["b"].data_ptr(), c["o"].data_ptr(), c["f"].data_ptr(), c["n"],
                                  self.all_freq, self.mode, self.T, c["base"], c["stride"],
                                  acc.data_ptr(), acc_obj.data_ptr(), ntok_acc.data_ptr(), s)

    def finalize(self, acc, acc_obj, ntok_acc):
        t = self.torch
        e = t.empty(self.dp.V, dtype=t.float32, device=self.dev)
        o = t.empty(1, dtype=t.float32, device=self.dev)
        nt = t.empty(1, dtype=t.int64, device=self.dev)
        s = t.cuda.current_stream(self.dev).cuda_stream
        self.dp.finalize_device(self.mode, self.T, acc.data_ptr(), acc_obj.data_ptr(), ntok_acc.data_ptr(),
                                e.data_ptr(), o.data_ptr(), nt.data_ptr(), s)
        return e, o, nt
