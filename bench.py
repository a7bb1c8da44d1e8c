"""Benchmark: batched unigram Viterbi Encode, 32k vocab, ~25-char sentences.

BASELINE.json config c2: 10M synthetic sentences (tools/synth.py, seed 1234 +
rank), 32k unigram model (data/synth32k_unigram.model), normalized bytes
resident in HBM before the timed region.  One step = one
spm_hip_encode_batch over the whole 10M-sentence batch (fast kernel, any
general-path re-runs, dense CSR compaction), exactly the C-ABI the drop-in
uses.  Multi-GPU: the corpus is sharded (each rank encodes its own 10M
sentences, no collective on the data path) → "scaling": "weak".

Prints ONE JSON line on rank 0 with `roofline` (the fast kernel, HIP-event
timed on the encode stream) and `cpu_baseline` (the CPU oracle port on a
bounded sample on this host's cores).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--sentences S]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sentencepiece-comments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sentences", type=int, default=10_000_000)
    ap.add_argument("--model", default=os.path.join(ROOT, "data", "synth32k_unigram.model"))
    ap.add_argument("--cpu-sample", type=int, default=2_000_000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--estep-sentences", type=int, default=100_000_000,
                    help="c4 corpus size per epoch (0 disables the E-step phase)")
    ap.add_argument("--estep-buffer", type=int, default=12_500_000,
                    help="synthetic sentences resident per rank (re-used to cover the shard)")
    ap.add_argument("--estep-epochs", type=int, default=3)
    ap.add_argument("--estep-warmup", type=int, default=1)
    ap.add_argument("--estep-cpu-sample", type=int, default=4_000_000)
    ap.add_argument("--raw-steps", type=int, default=5,
                    help="steps of the raw-text (device normalize + encode) phase; 0 disables")
    ap.add_argument("--train-lines", type=int, default=10_000_000,
                    help="c5: spm_train corpus size (0 disables the train phase; N=1 only)")
    ap.add_argument("--train-cpu-sample", type=int, default=200_000)
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r01o_pmc_unigram_fast.json"),
                    help="per-launch HBM traffic measured by rocprofv3 --pmc (optional)")
    return ap.parse_args()


def cpu_baseline(model_bytes, n, threads):
    """CPU oracle (restatement of unigram::Model::Encode) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    om = oracle_lib.OracleModel(model_bytes)
    buf, off = synth.normalized(n, seed=4321)
    t0 = time.perf_counter()
    om.encode_normalized_csr(buf, off, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "sentences/s", "cores": threads, "kind": "port",
            "sample": "%d synthetic normalized sentences (seed 4321), oracle/spm_oracle.cc "
                      "EncodeUnigram, %d threads, strided partition, %.1f s wall" % (n, threads, dt)}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    import spm_amd
    model_bytes = open(args.model, "rb").read()
    dm = spm_amd.DeviceModel(model_bytes)
    dm.set_timing(True)

    # Synthetic normalized corpus for this rank, resident in HBM.
    t0 = time.time()
    buf, off = synth.normalized(args.sentences, seed=1234 + rank)
    gen_s = time.time() - t0
    n = len(off) - 1
    total_bytes = int(off[-1])
    d_bytes = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_ids = torch.empty(max(total_bytes, 1), dtype=torch.int32, device=dev)
    d_tok = torch.empty(n + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def step():
        dm.encode_device(d_bytes.data_ptr(), d_off.data_ptr(), n, d_ids.data_ptr(),
                         d_tok.data_ptr(), stream=sp)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ntok = int(d_tok[-1].item())

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    fast_ms, gen_ms, general = [], [], 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        st = dm.stats()
        fast_ms.append(st.fast_kernel_ms)
        gen_ms.append(st.general_kernel_ms)
        general = st.general_path
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([float(n)], dtype=torch.float64, device=dev)
        dist.all_reduce(tot)
        total_sent = float(tot.item())
    else:
        total_sent = float(n)

    if rank == 0:
        ms_per_step = elapsed * 1000.0 / args.steps
        value = total_sent * args.steps / elapsed
        # Algorithmic bytes of one fast-kernel launch:
        # normalized bytes + offsets (8 B) read, ids (4 B/token) + ntok (4 B) written.
        algo_bytes = total_bytes + 8 * n + 4 * ntok + 4 * n
        k_ms = float(np.mean(fast_ms))
        info = dm.info()
        kernel_name = "unigram_fast_kernel<%d>" % (16 if info.max_piece_chars < 16 else 32
                                                   if info.max_piece_chars < 32 else 64) \
            if info.model_type == spm_amd.SPM_UNIGRAM else "bpe_half_kernel+bpe_fast_kernel"
        achieved = algo_bytes / (k_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.pmc_json):
            try:
                pmc = json.load(open(args.pmc_json))
                # Only a PMC summary of this very kernel counts.
                if pmc.get("kernel_substr", "") in kernel_name:
                    traffic = pmc.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": "sentences/sec Encode (32k unigram) @1 GPU" if info.model_type == spm_amd.SPM_UNIGRAM
                      else "sentences/sec Encode (32k BPE) @1 GPU",
            "value": value,
            "unit": "sentences/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/f32",
            "data": "synthetic",
            "config": {"workload": ("c2: batched unigram Viterbi Encode" if info.model_type == spm_amd.SPM_UNIGRAM
                                    else "c3: BPE Encode merge loop") +
                                   ", %d synthetic normalized sentences/GPU (mean %.2f B), 32k model %s"
                                   % (n, total_bytes / max(n, 1), os.path.relpath(args.model, ROOT)),
                       "sentences_per_gpu": n, "tokens_per_gpu": ntok,
                       "general_path_sentences": int(general),
                       "parallelism": "dp%d (sharded corpus, no collective)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kernel_name, "kernel_ms": k_ms,
                         "algo_bytes_per_launch": algo_bytes,
                         "general_kernel_ms": float(np.mean(gen_ms))},
            "synth_gen_s": gen_s,
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(model_bytes, args.cpu_sample,
                                                min(args.cpu_threads, os.cpu_count() or 1))
    # Release the encode buffers before the next phase.
    del d_bytes, d_off, d_ids, d_tok
    torch.cuda.empty_cache()
    if args.raw_steps > 0:
        e2e = raw_e2e_bench(args, dm, world, rank, dev, dist)
        if rank == 0:
            line["e2e_raw"] = e2e
    if args.estep_sentences > 0:
        es = estep_bench(args, model_bytes, world, rank, dev, dist)
        if rank == 0:
            line["estep"] = es
    if rank == 0 and world == 1 and args.train_lines > 0:
        line["train"] = train_bench(args)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def train_bench(args):
    """c5: full `spm_train --model_type=unigram --vocab_size=32000` (lib/spm_train:
    device seed mining, device E-steps in PARITY mode with 16 buckets, device
    pruning Viterbi) on a synthetic corpus file of --train-lines lines.  One
    run = the whole training, file read to .model/.vocab written.  The CPU
    baseline is the oracle trainer (oracle/spm_oracle_train.inc, single-thread
    seed mining, 16-bucket threaded E-step) on a bounded sample, with the GPU
    trainer timed on the same sample beside it."""
    import subprocess
    import tempfile
    import train_bench as tb
    d = tempfile.mkdtemp(prefix="spm_c5_")
    spec = "--normalization_rule_name=identity --num_threads=16"

    def run(lines, tag):
        corpus = os.path.join(d, tag + ".txt")
        tb.write_corpus(corpus, lines, 1234)
        cmd = [tb.TRAIN, "--input=" + corpus, "--model_prefix=" + os.path.join(d, tag),
               "--model_type=unigram", "--vocab_size=32000", "--timings"] + spec.split()
        t0 = time.perf_counter()
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        wall = time.perf_counter() - t0
        if p.returncode != 0:
            raise RuntimeError(p.stderr.decode(errors="replace")[-2000:])
        tm = json.loads(p.stdout.decode().strip().splitlines()[-1])
        tm["process_wall_s"] = wall
        return corpus, tm

    _, tm = run(args.train_lines, "main")
    res = {"metric": "spm_train unigram 32k end-to-end @1 GPU", "value": tm["total_s"], "unit": "s",
           "higher_is_better": False, "lines": args.train_lines, "stages": tm,
           "workload": "c5: spm_train --model_type=unigram --vocab_size=32000 %s on %d synthetic "
                       "lines (tools/synth.py raw text), file read to .model written" % (spec, args.train_lines)}
    if not args.no_cpu_baseline and args.train_cpu_sample > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        corpus, gtm = run(args.train_cpu_sample, "sample")
        lines = oracle_lib.read_lines_binary(corpus)
        t0 = time.perf_counter()
        ot = oracle_lib.OracleTrainer("--vocab_size=32000 " + spec, lines)
        ot.train()
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": dt, "unit": "s", "cores": 16, "kind": "port",
                               "sample": "%d lines of the same generator; oracle trainer (single-thread "
                                         "load/seed/prune, 16-bucket threaded E-step) %.1f s vs "
                                         "lib/spm_train %.2f s on the same sample"
                                         % (args.train_cpu_sample, dt, gtm["total_s"]),
                               "gpu_same_sample_s": gtm["total_s"]}
    return res


def raw_e2e_bench(args, dm, world, rank, dev, dist):
    """Raw text → ids on the device: the same 10M-sentence corpus as c2 but as
    RAW lines resident in HBM; one step = spm_hip_normalize_batch_device
    (Normalizer::Normalize with the model's nmt_nfkc charsmap: length pass,
    scan, write pass) + spm_hip_encode_batch + spm_hip_finalize_ids (the
    unk-run merge of PopulateSentencePieceText), i.e. the whole
    SentencePieceProcessor::Encode(ids) per line.  Weak-scaled like c2."""
    import ctypes
    import torch
    buf, off = synth.raw(args.sentences, seed=1234 + rank)
    n = len(off) - 1
    d_in = torch.from_numpy(buf).to(dev)
    d_in_off = torch.from_numpy(off.view(np.int64)).to(dev)
    cap = int(off[-1]) * 2 + 4 * n
    d_norm = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_noff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    d_tok = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_fin = torch.empty(cap, dtype=torch.int32, device=dev)
    d_fin_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    L = dm._L
    tot = ctypes.c_uint64()

    def step():
        rc = L.spm_hip_normalize_batch_device(dm.h, d_in.data_ptr(), d_in_off.data_ptr(), n,
                                              d_norm.data_ptr(), cap, d_noff.data_ptr(),
                                              ctypes.byref(tot), sp)
        if rc != 0:
            raise RuntimeError("normalize_device failed: %d" % rc)
        dm.encode_device(d_norm.data_ptr(), d_noff.data_ptr(), n, d_ids.data_ptr(), d_tok.data_ptr(),
                         stream=sp)
        # Id epilogue (unk-run merge; no extra options) → final Encode(ids).
        dm.finalize_ids_device("", d_ids.data_ptr(), d_tok.data_ptr(), n, d_fin.data_ptr(), cap,
                               d_fin_off.data_ptr(), stream=sp)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.raw_steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return {"metric": "sentences/sec raw text -> ids (device Normalize + Encode + id epilogue) @%d GPU" % world,
            "value": n * world * args.raw_steps / el, "unit": "sentences/s", "steps": args.raw_steps,
            "ms_per_step": el * 1000.0 / args.raw_steps, "raw_bytes_per_gpu": int(off[-1]),
            "normalized_bytes_per_gpu": int(tot.value),
            "workload": "%d raw synthetic lines/GPU resident in HBM (mean %.2f B), model %s (nmt_nfkc)"
                        % (n, int(off[-1]) / max(n, 1), os.path.relpath(args.model, ROOT))}


def estep_bench(args, model_bytes, world, rank, dev, dist):
    """c4: unigram trainer E-step over a fixed corpus (default 100M synthetic
    normalized sentences, freq 1, no whitespace split) sharded over the ranks
    (strong scaling), pieces = the NORMAL pieces of the 32k model.  One epoch =
    accumulate on every rank + one RCCL SUM all-reduce of the fp64 expected
    counts + finalize."""
    import torch
    import dist_estep
    import spm_amd
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import model_reader
    pcs = [(p, s) for p, s, t in model_reader.read_pieces(model_bytes) if t == 1]
    pieces = [p for p, _ in pcs]
    scores = np.array([s for _, s in pcs], dtype=np.float32)
    dp = spm_amd.DevicePieces(pieces, scores)
    total = args.estep_sentences
    lo, hi = dist_estep.contiguous_shard(total, world, rank)
    mine = hi - lo
    m = min(mine, args.estep_buffer)
    buf, off = synth.normalized(m, seed=99 + rank)
    d_b = torch.from_numpy(buf).to(dev)
    d_o = torch.from_numpy(off.view(np.int64)).to(dev)
    d_f = torch.ones(m, dtype=torch.int64, device=dev)
    runner = dist_estep.DeviceEStep(dp, dist_estep.FAST, 1, dev, total)
    chunks = []
    left = mine
    while left > 0:
        k = min(left, m)
        chunks.append({"b": d_b, "o": d_o, "f": d_f, "n": k, "base": lo + mine - left, "stride": 1})
        left -= k
    ar = (lambda x: dist.all_reduce(x)) if world > 1 else None

    def epoch():
        return dist_estep.run_sharded(chunks, dist_estep.FAST, 1, dp.V, runner.accumulate, runner.finalize,
                                      runner.make_zeros, all_reduce=ar)

    for _ in range(args.estep_warmup):
        epoch()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.estep_epochs):
        e, o, nt = epoch()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    sec = el / args.estep_epochs
    res = {"metric": "E-step sec/epoch @%d GPU" % world, "value": sec, "unit": "s/epoch",
           "higher_is_better": False, "n_gpus": world, "epochs": args.estep_epochs,
           "sentences_per_epoch": total, "sentences_per_s": total / sec, "mode": "FAST (fp64 accumulate)",
           "pieces": dp.V, "ntok": int(nt.item()), "obj": float(o.item()),
           "workload": "c4: %d synthetic normalized sentences/epoch (freq 1, no whitespace split), "
                       "NORMAL pieces of data/synth32k_unigram.model, sharded over %d rank(s), one "
                       "RCCL all-reduce of fp64[V] per epoch" % (total, world)}
    if rank == 0 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        ns = args.estep_cpu_sample
        bb, oo = synth.normalized(ns, seed=7)
        b = bb.tobytes()
        sents = [b[int(oo[i]):int(oo[i + 1])] for i in range(ns)]
        th = min(args.cpu_threads, os.cpu_count() or 1)
        t0 = time.perf_counter()
        oracle_lib.estep(sents, np.ones(ns, dtype=np.int64), pieces, scores, th)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": total * dt / ns, "unit": "s/epoch (extrapolated)", "cores": th,
                               "kind": "port", "sample": "%d sentences, oracle RunEStep emulation with %d "
                               "threads, %.1f s wall, extrapolated to %d sentences" % (ns, th, dt, total)}
    return res


if __name__ == "__main__":
    main()
