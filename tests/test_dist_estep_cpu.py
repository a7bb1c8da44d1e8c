"""World-size-2 gloo test of the sharded E-step driver (dist_estep.py) on CPU.

Each rank accumulates its shard with the oracle's partial E-step (the same
contract as spm_hip_estep_accumulate), the accumulators are SUM-all-reduced
over gloo and finalized; rank 0 checks the result against the single-process
oracle RunEStep at num_threads = T.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dist_estep as D
import model_reader
import oracle_lib as O
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup():
    mb = open(os.path.join(ROOT, "tests", "golden", "test_model.model"), "rb").read()
    pcs = [(p, s) for p, s, t in model_reader.read_pieces(mb) if t == 1]
    pieces = [p for p, _ in pcs]
    scores = np.array([s for _, s in pcs], dtype=np.float32)
    buf, off = synth.normalized(3000, seed=3)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(3000)]
    freqs = np.arange(3000) % 4 + 1
    return pieces, scores, sents, freqs


def _all_gather(x):
    out = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(out, x)
    return out


def _worker(rank, world, port, mode, T, out, gather=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pieces, scores, sents, freqs = _setup()
    V = len(pieces)
    all_freq = int(freqs.sum())
    chunks = D.plan_chunks(sents, freqs, mode, T, world, rank)

    def acc_fn(c, acc, acc_obj, ntok_acc):
        s, f, base, stride = c
        O.estep_partial(s, f, pieces, scores, all_freq, mode, T, base, stride,
                        acc.numpy(), acc_obj.numpy(), ntok_acc.numpy())

    def zeros(shape, dtype):
        return torch.from_numpy(np.zeros(shape, dtype=dtype))

    def fin(acc, acc_obj, ntok_acc):
        return D.finalize_host(mode, T, V, acc.numpy(), acc_obj.numpy(), ntok_acc.numpy())

    e, obj, nt = D.run_sharded(chunks, mode, T, V, acc_fn, fin, zeros, all_reduce=dist.all_reduce,
                               all_gather=_all_gather if gather else None, world=world, rank=rank)
    if rank == 0:
        out.put((e, obj, nt))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode,T,gather", [(D.PARITY, 4, False), (D.PARITY, 3, False), (D.FAST, 1, False),
                                           (D.PARITY, 4, True), (D.PARITY, 3, True)])
def test_sharded_estep_gloo_world2(mode, T, gather):
    """gather: PARITY rows moved by one all-gather of each rank's owned rows
    (dist_estep.gather_owned_rows) instead of the zero-padded SUM all-reduce."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, mode, T, q, gather)) for r in range(2)]
    for p in ps:
        p.start()
    e, obj, nt = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    pieces, scores, sents, freqs = _setup()
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, T)
    assert nt == nt_ref
    if mode == D.PARITY:
        assert np.array_equal(e, e_ref)       # bit-exact at num_threads = T
        assert obj == obj_ref
    else:
        nz = e_ref != 0
        assert np.max(np.abs(e - e_ref)[nz] / e_ref[nz]) < 1e-3


@pytest.mark.parametrize("mode,T", [(D.PARITY, 1), (D.PARITY, 3), (D.PARITY, 8), (D.PARITY, 16), (D.FAST, 1)])
def test_cxx_shard_plan_injected_sum(mode, T):
    """The C++ shard plan spm_train --num_gpus uses (csrc/shard_plan.h through
    spm_hip_estep_shard_plan): every rank accumulates its segments with the
    oracle's partial E-step (the spm_hip_estep_accumulate contract), the rank
    accumulators are summed in rank order in process (the reduction the
    trainer does over RCCL or the host), and the result equals the world-1
    RunEStep at num_threads = T bit for bit (PARITY) for W = 1..8."""
    import spm_amd as S
    pieces, scores, sents, freqs = _setup()
    V = len(pieces)
    all_freq = int(freqs.sum())
    n = len(sents)
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, T)
    for W in (1, 2, 3, 4, 5, 8):
        seen = np.zeros(n, dtype=np.int64)
        shapes = D.accumulator_shapes(mode, T, V)
        tot = [np.zeros(sh, dtype=dt) for sh, dt in shapes]
        owner = np.full(T, -1)
        for r in range(W):
            acc = [np.zeros(sh, dtype=dt) for sh, dt in shapes]
            for base, stride, count in S.estep_shard_plan(n, mode, T, W, r):
                idx = base + stride * np.arange(count, dtype=np.int64)
                seen[idx] += 1
                if mode == D.PARITY:  # a bucket lives on one rank only
                    for b in np.unique(idx % T):
                        assert owner[b] in (-1, r)
                        owner[b] = r
                O.estep_partial([sents[i] for i in idx], freqs[idx], pieces, scores, all_freq, mode, T,
                                base, stride, acc[0], acc[1], acc[2])
            for t, a in zip(tot, acc):
                t += a
        assert np.all(seen == 1), "plan must cover every sentence once (W=%d)" % W
        if mode == D.PARITY:
            # The row each rank's reduction gathers (trainer ReduceToRank0,
            # both the RCCL send/recv and the host-copy branch) comes from the
            # rank the plan gave the bucket to; so does the Python gather.
            for b in range(T):
                assert S.estep_bucket_owner(b, T, W) == owner[b], (b, T, W)
                assert b in D.owned_buckets(T, W, int(owner[b]))
        e, obj, nt = D.finalize_host(mode, T, V, tot[0], tot[1], tot[2])
        assert nt == nt_ref
        if mode == D.PARITY:
            assert np.array_equal(e, e_ref), W
            assert obj == obj_ref
        else:
            nz = e_ref != 0
            assert np.max(np.abs(e - e_ref)[nz] / e_ref[nz]) < 1e-3


def _epoch_worker(rank, world, port, mode, T, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pieces, scores, sents, freqs = _setup()
    V = len(pieces)
    all_freq = int(freqs.sum())
    chunks = D.plan_chunks(sents, freqs, mode, T, world, rank)

    def acc_fn(c, acc, acc_obj, ntok_acc):
        s, f, base, stride = c
        O.estep_partial(s, f, pieces, scores, all_freq, mode, T, base, stride,
                        acc.numpy(), acc_obj.numpy(), ntok_acc.numpy())

    def zeros(shape, dtype):
        return torch.from_numpy(np.zeros(shape, dtype=dtype))

    def fin(acc, acc_obj, ntok_acc):
        return D.finalize_host(mode, T, V, acc.numpy(), acc_obj.numpy(), ntok_acc.numpy())

    import time
    epoch = D.make_epoch(chunks, mode, T, V, acc_fn, fin, zeros, world=world, rank=rank,
                         all_reduce=dist.all_reduce, all_gather=_all_gather, clock=time.perf_counter)
    times = {}
    e, obj, nt = epoch(times)
    if rank == 0:
        out.put((e, obj, nt, times))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,T", [(D.PARITY, 16), (D.PARITY, 3), (D.FAST, 1)])
def test_bench_epoch_driver_gloo_world2(mode, T):
    """The epoch bench.py's E-step leg runs (dist_estep.make_epoch): at world 2
    PARITY takes the owned-row all-gather path, FAST the SUM
    all-reduce, the per-rank compute / collective split is filled in, and the
    result equals the single-process RunEStep emulation (PARITY bit for bit)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_epoch_worker, args=(r, 2, port, mode, T, q)) for r in range(2)]
    for p in ps:
        p.start()
    e, obj, nt, times = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert times["path"] == ("gather" if mode == D.PARITY else "allreduce")
    assert times["compute_s"] > 0 and times["collective_s"] >= 0
    pieces, scores, sents, freqs = _setup()
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, T)
    assert nt == nt_ref
    if mode == D.PARITY:
        assert np.array_equal(e, e_ref) and obj == obj_ref
    else:
        nz = e_ref != 0
        assert np.max(np.abs(e - e_ref)[nz] / e_ref[nz]) < 1e-3


def test_cxx_bucket_owner_bounds():
    """spm_hip_estep_bucket_owner rejects buckets outside [0, T) and bad
    world/thread counts; with W > T ranks >= T own nothing."""
    import spm_amd as S
    assert S.estep_bucket_owner(-1, 4, 2) == -1
    assert S.estep_bucket_owner(4, 4, 2) == -1
    assert S.estep_bucket_owner(0, 0, 2) == -1
    assert S.estep_bucket_owner(0, 4, 0) == -1
    assert [S.estep_bucket_owner(b, 3, 8) for b in range(3)] == [0, 1, 2]
    assert [S.estep_bucket_owner(b, 5, 2) for b in range(5)] == [0, 1, 0, 1, 0]
