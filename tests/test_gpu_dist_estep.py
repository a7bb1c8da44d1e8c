"""The sharded E-step driver (dist_estep.run_sharded) with the DEVICE
accumulate (dist_estep.DeviceEStep -> spm_hip_estep_accumulate /
spm_hip_estep_finalize) under a real world-2 process group: two processes on
one GPU, gloo collectives (host copies of the device accumulators; the
8-GPU driver runs the same calls over RCCL).  Rank 0's result must equal the
single-process oracle RunEStep at num_threads = T bit for bit (PARITY),
including the owned-row gather."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _setup():
    import model_reader
    import synth
    mb = open(os.path.join(ROOT, "tests", "golden", "test_model.model"), "rb").read()
    pcs = [(p, s) for p, s, t in model_reader.read_pieces(mb) if t == 1]
    pieces = [p for p, _ in pcs]
    scores = np.array([s for _, s in pcs], dtype=np.float32)
    buf, off = synth.normalized(6000, seed=5)
    b = buf.tobytes()
    sents = [b[int(off[i]):int(off[i + 1])] for i in range(6000)]
    freqs = np.arange(6000) % 3 + 1
    return pieces, scores, sents, freqs


def _worker(rank, world, port, mode, T, gather, out):
    import sys
    for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "sentencepiece-comments_amd"),
              os.path.join(ROOT, "tools")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import dist_estep as D
    import spm_amd as S
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    pieces, scores, sents, freqs = _setup()
    dp = S.DevicePieces(pieces, scores)
    runner = D.DeviceEStep(dp, mode, T, dev, int(freqs.sum()))
    chunks = [runner.upload(s, f, base, stride)
              for s, f, base, stride in D.plan_chunks(sents, freqs, mode, T, world, rank)]

    def all_reduce(x):  # gloo on host copies of the device tensor
        torch.cuda.synchronize(dev)
        h = x.cpu()
        dist.all_reduce(h)
        x.copy_(h.to(dev))

    def all_gather(x):
        torch.cuda.synchronize(dev)
        h = x.cpu()
        outs = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(outs, h)
        return [o.to(dev) for o in outs]

    e, o, nt = D.run_sharded(chunks, mode, T, dp.V, runner.accumulate, runner.finalize, runner.make_zeros,
                             all_reduce=all_reduce, all_gather=all_gather if gather else None,
                             world=world, rank=rank, sync=runner.sync)
    torch.cuda.synchronize(dev)
    if rank == 0:
        out.put((e.cpu().numpy(), float(o.item()), int(nt.item())))
    dp.close()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode,T,gather", [(1, 4, True), (1, 3, True), (1, 4, False), (0, 1, False)])
def test_device_estep_sharded_world2(mode, T, gather):
    import torch.multiprocessing as mp
    import oracle_lib as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, mode, T, gather, q)) for r in range(2)]
    for p in ps:
        p.start()
    e, obj, nt = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    pieces, scores, sents, freqs = _setup()
    e_ref, obj_ref, nt_ref = O.estep(sents, freqs, pieces, scores, T)
    assert nt == nt_ref
    if mode == 1:
        assert np.array_equal(e.view(np.uint32), np.asarray(e_ref, dtype=np.float32).view(np.uint32))
        assert obj == obj_ref
    else:
        nz = e_ref != 0
        assert np.max(np.abs(e - e_ref)[nz] / e_ref[nz]) < 1e-3
