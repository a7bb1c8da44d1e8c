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
           A row has exactly one owner, so the rows are GATHERED (one
           all-gather of each rank's ceil(T/W) packed rows, no arithmetic on
           them; 1/W of a zero-padded SUM all-reduce's payload) and obj[T] /
           ntok[T] SUM-reduced (exact: one non-zero contributor per entry);
           finalize sums the buckets in order 0..T-1, bit-equal to the
           reference at num_threads = T.

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


def gather_owned_rows(acc, T, V, world, rank, all_gather):
    """PARITY rows to every rank without arithmetic: this rank packs the rows
    it owns (b % world == rank) into a [ceil(T/world), V] block, one
    all_gather(block) -> [block of rank 0, ..., block of rank world-1]
    collects them, and the [T, V] accumulator is reassembled in bucket order."""
    R = (T + world - 1) // world
    rows = acc.view(T, V)
    mine = acc.new_zeros((R, V))
    for k, b in enumerate(owned_buckets(T, world, rank)):
        mine[k] = rows[b]
    blocks = all_gather(mine)
    for r in range(world):
        for k, b in enumerate(owned_buckets(T, world, r)):
            rows[b] = blocks[r][k]


def run_sharded(chunks, mode, T, V, accumulate, finalize, make_zeros, all_reduce=None, all_gather=None,
                world=1, rank=0, sync=None, clock=None, times=None):
    """Generic driver.  accumulate(chunk, acc, acc_obj, ntok_acc); all_reduce(x)
    sums a buffer in place across ranks (None for a single process);
    all_gather(x) returns the list of every rank's x (PARITY rows; without it
    PARITY falls back to the exact zero-padded SUM all-reduce); sync() makes
    the accumulators complete after accumulate calls that deferred their
    folds (DeviceEStep).  clock() (device-synchronizing timestamp) and a
    `times` dict attribute this rank's time: times["compute_s"] (accumulate +
    sync), times["collective_s"] (row gather / all-reduces), times["path"]
    ("gather" | "allreduce" | "none") are added to."""
    (sa, da), (so, do), (sn, dn) = accumulator_shapes(mode, T, V)
    acc, acc_obj, ntok_acc = make_zeros(sa, da), make_zeros(so, do), make_zeros(sn, dn)
    t0 = clock() if clock else 0.0
    for c in chunks:
        accumulate(c, acc, acc_obj, ntok_acc)
    if sync is not None:
        sync()
    t1 = clock() if clock else 0.0
    path = "none"
    if all_reduce is not None:
        if mode == PARITY and all_gather is not None:
            gather_owned_rows(acc, T, V, world, rank, all_gather)
            path = "gather"
        else:
            all_reduce(acc)
            path = "allreduce"
        all_reduce(acc_obj)
        all_reduce(ntok_acc)
    t2 = clock() if clock else 0.0
    if times is not None:
        times["compute_s"] = times.get("compute_s", 0.0) + (t1 - t0)
        times["collective_s"] = times.get("collective_s", 0.0) + (t2 - t1)
        times["path"] = path
    return finalize(acc, acc_obj, ntok_acc)


def make_epoch(chunks, mode, T, V, accumulate, finalize, make_zeros, world=1, rank=0, all_reduce=None,
               all_gather=None, sync=None, clock=None):
    """One EM sub-iteration's E-step over this rank's chunks, as bench.py and
    any multi-GPU caller run it: at world > 1 PARITY moves its bucket rows
    with all_gather (gather_owned_rows, every row has one owner) and FAST
    SUM-all-reduces fp64[V]; a single process runs no collective.  The
    returned epoch(times=None) attributes this rank's time into `times`
    (compute_s, collective_s, path) when given, using clock()."""
    def epoch(times=None):
        return run_sharded(chunks, mode, T, V, accumulate, finalize, make_zeros,
                           all_reduce=all_reduce if world > 1 else None,
                           all_gather=all_gather if (world > 1 and mode == PARITY) else None,
                           world=world, rank=rank, sync=sync,
                           clock=clock if times is not None else None, times=times)
    return epoch


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
        """Deferred folds (SPM_ESTEP_DEFER_FOLD): a call's last PARITY fold
        overlaps the next call's walks; sync() / finalize() complete them."""
        s = self.torch.cuda.current_stream(self.dev).cuda_stream
        self.dp.accumulate_device(c["b"].data_ptr(), c["o"].data_ptr(), c["f"].data_ptr(), c["n"],
                                  self.all_freq, self.mode, self.T, c["base"], c["stride"],
                                  acc.data_ptr(), acc_obj.data_ptr(), ntok_acc.data_ptr(), s, defer=True)

    def sync(self):
        self.dp.sync_device(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def finalize(self, acc, acc_obj, ntok_acc):
        t = self.torch
        e = t.empty(self.dp.V, dtype=t.float32, device=self.dev)
        o = t.empty(1, dtype=t.float32, device=self.dev)
        nt = t.empty(1, dtype=t.int64, device=self.dev)
        s = t.cuda.current_stream(self.dev).cuda_stream
        self.dp.finalize_device(self.mode, self.T, acc.data_ptr(), acc_obj.data_ptr(), ntok_acc.data_ptr(),
                                e.data_ptr(), o.data_ptr(), nt.data_ptr(), s)
        return e, o, nt
