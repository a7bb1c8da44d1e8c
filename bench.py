"""Benchmark: batched unigram Viterbi Encode, 32k vocab, ~25-char sentences.

BASELINE.json config c2: 10M synthetic sentences (tools/synth.py, seed 1234 +
rank), 32k unigram model (data/synth32k_unigram.model), normalized bytes
resident in HBM before the timed region.  One step = one
spm_hip_encode_batch over the whole 10M-sentence batch (fast kernel, any
general-path re-runs, dense CSR compaction), exactly the C-ABI the drop-in
uses.  Multi-GPU: the corpus is sharded (each rank encodes its own 10M
sentences, no collective on the data path) → "scaling": "weak".

Prints ONE JSON line on rank 0 with `roofline` (the fast kernel, HIP-event
timed on the encode stream, plus the trie-probe rate), `cpu_baseline` (the
CPU oracle port on a bounded sample, 16 threads = the GPU box's CPU share,
and 1 thread) and the other legs: `bpe_c3` (c3, its own roofline),
`e2e_raw` (raw text → final ids), `estep` (c4, PARITY mode), `latency`,
`train` (c5) and `train_bpe` (N=1 only).  The line keeps the numbers (about
5 KB, ending with a `legs` summary: value, roofline frac and PMC traffic per
leg); notes, logs and per-batch tables go to the --detail side file.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--sentences S]

`--gpus N` with N > 1 outside torchrun starts N worker processes (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1) before anything touches the
GPU and prints rank 0's line; under torchrun the env is used as given.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sentencepiece-comments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

_T0 = time.time()


def log(msg):
    """Progress on stderr (a run silent for minutes looks hung to the harness)."""
    sys.stderr.write("[bench %6.1fs] %s\n" % (time.time() - _T0, msg))
    sys.stderr.flush()


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BOX_CPU_SHARE = 16     # CPU threads of one GPU's share of the box


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sentences", type=int, default=10_000_000)
    ap.add_argument("--model", default=os.path.join(ROOT, "data", "synth32k_unigram.model"))
    ap.add_argument("--bpe-model", default=os.path.join(ROOT, "data", "synth32k_bpe.model"))
    ap.add_argument("--bpe-steps", type=int, default=5, help="c3 BPE leg steps (0 disables)")
    ap.add_argument("--cpu-sample", type=int, default=2_000_000)
    ap.add_argument("--cpu-sample-1t", type=int, default=500_000)
    ap.add_argument("--cpu-threads", type=int, default=BOX_CPU_SHARE)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--estep-sentences", type=int, default=100_000_000,
                    help="c4 corpus size per epoch (0 disables the E-step phase)")
    ap.add_argument("--estep-buffer", type=int, default=12_500_000,
                    help="synthetic sentences resident per rank (re-used to cover the shard)")
    ap.add_argument("--estep-warmup", type=int, default=1)
    ap.add_argument("--estep-parity-epochs", type=int, default=3,
                    help="PARITY-mode epochs (T = --estep-threads buckets); 0 disables")
    ap.add_argument("--estep-threads", type=int, default=16)
    ap.add_argument("--estep-cpu-sample", type=int, default=4_000_000)
    ap.add_argument("--raw-steps", type=int, default=5,
                    help="steps of the raw-text (device normalize + encode) phase; 0 disables")
    ap.add_argument("--train-lines", type=int, default=100_000_000,
                    help="c5: spm_train corpus size (0 disables the train phase; N=1 only)")
    ap.add_argument("--bpe-train-lines", type=int, default=10_000_000,
                    help="BPE trainer leg corpus size (0 disables; N=1 only)")
    ap.add_argument("--train-cpu-sample", type=int, default=200_000)
    ap.add_argument("--ja-lines", type=int, default=1_000_000,
                    help="multi-byte leg: wagahaiwa lines repeated to at least this many (0 disables)")
    ap.add_argument("--latency-calls", type=int, default=2000,
                    help="single-sentence / small-batch latency leg (lib/spm_latency) calls; 0 disables")
    ap.add_argument("--no-probe-stats", action="store_true")
    ap.add_argument("--no-parity-check", action="store_true",
                    help="skip the full-size checks of the benchmarked outputs against the CPU oracle")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU check of the launcher: gloo process group, no GPU work; prints the "
                         "line skeleton with n_gpus and the summed per-rank sentence counts")
    ap.add_argument("--pmc-dir", default=os.path.join(ROOT, "profiles", "pmc"),
                    help="stamped PMC summaries of the shipped kernels (tools/pmc_traffic.py, "
                         "tools/gpu_r06_pmc.sh): a summary counts only when its source stamp matches")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="side file for the full per-leg record (notes, logs, per-batch tables); the "
                         "printed line keeps the numbers")
    return ap.parse_args(argv)


def launch_workers(args):
    """--gpus N outside torchrun: N children, one per GPU, started before any
    GPU call in this process; rank 0's JSON line is forwarded."""
    n = args.gpus
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].communicate()[0].decode()
    rc = max(abs(p.wait()) for p in procs)
    # Only the JSON line (backends may chat on stdout).
    sys.stdout.write("".join(l + "\n" for l in out.splitlines() if l.startswith("{")))
    sys.stdout.flush()
    return rc


ENCODE_PMC_LEGS = ("c2", "c3", "ja", "ja_coop")


def pmc_traffic(pmc_dir, leg, kernels, launches=None):
    """HBM bytes per launch of `kernels` (kernel-name substrings) on bench leg
    `leg`, summed, from the stamped PMC summaries in pmc_dir
    (tools/pmc_traffic.py writes <leg>__<kernel>.json).  A summary counts only
    when its `src_sha` equals the stamp of the kernel sources this run loads
    (pmc_stamp.src_sha256): a stale summary gives traffic null and says why.
    launches: per-kernel dispatch count per bench launch (default 1 each).
    Encode legs average the timed launches only: their last dispatch is the
    blocking call after the timed region, which also writes piece lengths."""
    import pmc_stamp
    want = pmc_stamp.src_sha256()
    tot, srcs, why = 0.0, [], []
    for k, kern in enumerate(kernels):
        path = os.path.join(pmc_dir, "%s__%s.json" % (leg, pmc_stamp.slug(kern)))
        if not os.path.exists(path):
            why.append("no summary %s" % os.path.relpath(path, ROOT))
            continue
        pmc = json.load(open(path))
        if pmc.get("src_sha") != want:
            why.append("%s stamped %s, sources %s" % (os.path.basename(path), str(pmc.get("src_sha"))[:12],
                                                      want[:12]))
            continue
        per = pmc_stamp.steady_bytes(pmc, drop_last=leg in ENCODE_PMC_LEGS)
        tot += per * (launches[k] if launches else 1)
        srcs.append(os.path.relpath(path, ROOT))
    if why:
        return None, {"traffic_note": "; ".join(why)}
    return int(round(tot)), {"traffic_source": srcs, "traffic_stamp": want[:16]}


def cpu_encode_baseline(model_bytes, n, threads):
    """CPU oracle (restatement of unigram::Model::Encode / bpe::Model::Encode)
    on a bounded sample (test infrastructure: timed only, never shipped)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    import synth
    om = oracle_lib.OracleModel(model_bytes)
    buf, off = synth.normalized(n, seed=4321)
    t0 = time.perf_counter()
    om.encode_normalized_csr(buf, off, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "sentences/s", "cores": threads, "kind": "port",
            "sample": "%d synthetic normalized sentences (seed 4321), oracle/spm_oracle.cc Encode, "
                      "%d thread(s), strided partition, %.1f s wall" % (n, threads, dt)}


class ParityError(RuntimeError):
    pass


def encode_mismatches(ids, to, ref_ids, ref_to, lens=None, ref_lens=None):
    """Sentences whose (ids[, piece byte lengths]) differ between two CSR
    outputs; 0 when the whole arrays are equal (the normal case, one compare)."""
    import numpy as np
    to = np.asarray(to).astype(np.uint64)
    ref_to = np.asarray(ref_to).astype(np.uint64)
    same_to = np.array_equal(to, ref_to)
    if same_to and np.array_equal(ids, ref_ids) and (lens is None or np.array_equal(lens, ref_lens)):
        return 0
    n = len(to) - 1
    bad = 0
    for i in range(n):
        a, b, c, d = int(to[i]), int(to[i + 1]), int(ref_to[i]), int(ref_to[i + 1])
        if (b - a != d - c or not np.array_equal(ids[a:b], ref_ids[c:d]) or
                (lens is not None and not np.array_equal(lens[a:b], ref_lens[c:d]))):
            bad += 1
    return bad


def parity_encode(model_bytes, buf, off, ids, lens, to, threads, period=None):
    """Full-size check of one benchmarked encode (all of this rank's
    sentences) against the CPU oracle (oracle/spm_oracle.cc, test
    infrastructure used here only as the checker, outside the timed region).
    period = p: the corpus is its first p sentences repeated; the oracle
    encodes those once and its output, repeated, is the expected output of
    every sentence."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    om = oracle_lib.OracleModel(model_bytes)
    t0 = time.perf_counter()
    if period:
        n = len(off) - 1
        reps = (n + period - 1) // period
        uoff = off[:period + 1].copy()
        u_ids, u_lens, u_to = om.encode_normalized_csr(buf[:int(uoff[-1])], uoff, threads=threads, with_lens=True)
        cnt = np.tile((u_to[1:] - u_to[:-1]).astype(np.uint64), reps)[:n]
        rto = np.zeros(n + 1, dtype=np.uint64)
        rto[1:] = np.cumsum(cnt, dtype=np.uint64)
        rids = np.tile(u_ids, reps)[:int(rto[-1])]
        rlens = np.tile(u_lens, reps)[:int(rto[-1])]
    else:
        rids, rlens, rto = om.encode_normalized_csr(buf, off, threads=threads, with_lens=True)
    dt = time.perf_counter() - t0
    bad = encode_mismatches(ids, to, rids, rto, lens, rlens)
    return {"sentences": len(off) - 1, "tokens": int(rto[-1]), "mismatches": bad,
            "compared": "token ids and piece byte lengths of every sentence (timed step's ids, lengths "
                        "from one more call) vs oracle Encode" +
                        (" (the corpus repeats its first %d sentences: oracle output of those, repeated)" % period
                         if period else ""),
            "oracle_s": dt, "oracle_threads": threads}


def parity_estep(args, buf, off, total, pieces, scores, T, e, obj, ntok):
    """Full-size check of the last timed PARITY epoch (expected[V], obj, ntok
    over all `total` sentences, sentence g = resident buffer[g mod m]) against
    the oracle's RunEStep emulation with T buckets, bit for bit."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    m = len(off) - 1
    th = min(args.cpu_threads, os.cpu_count() or 1)
    log("c4 PARITY full-size oracle check (%d sentences, %d threads)" % (total, th))
    t0 = time.perf_counter()
    re, ro, rn = oracle_lib.estep_cyclic_csr(buf, off, np.ones(m, dtype=np.int64), total, pieces, scores, T)
    dt = time.perf_counter() - t0
    got = e.cpu().numpy()
    bad = int(np.count_nonzero(got.view(np.uint32) != re.view(np.uint32)))
    obj_eq = bool(np.float32(obj).view(np.uint32) == np.float32(ro).view(np.uint32))
    res = {"sentences": total, "pieces": len(pieces), "mismatches": bad + (0 if obj_eq else 1) + (0 if ntok == rn else 1),
           "expected_mismatches": bad, "obj_equal": obj_eq, "ntok_equal": ntok == rn,
           "compared": "expected[V] float bits, obj float bits and ntok of the last timed epoch vs the "
                       "oracle RunEStep emulation (T=%d buckets) over the same sentence sequence" % T,
           "oracle_s": dt, "oracle_threads": T}
    if bad:
        idx = np.nonzero(got.view(np.uint32) != re.view(np.uint32))[0][:5]
        res["first"] = [(int(i), float(got[i]), float(re[i])) for i in idx]
    return res


def kernel_label(info, spm_amd):
    if info.model_type != spm_amd.SPM_UNIGRAM:
        # csrc/bpe_kernels.hip: one sentence per lane while piece ids fit int16
        return ("bpe_lane_kernel+bpe_fast_kernel+bpe_compact_kernel" if info.piece_size < 32768
                else "bpe_half_kernel+bpe_fast_kernel+bpe_compact_kernel")
    if info.fast_variant == 0:
        return "unigram_general_kernel"
    # spm_hip_model_info.fast_variant: 1 byte kernel, 2 char kernel, 3 wide-char kernel (csrc/unigram_encode.hip)
    if info.fast_variant == 3:
        return "unigram_fast_kernel<16, false, 3, false, true>"
    return "unigram_fast_kernel<%d, %s>" % (info.ring_width, "true" if info.fast_variant == 1 else "false")


# PMC kernel sets per leg: the kernels inside the leg's HIP-event span.
PMC_KERNELS = {"c2": ["unigram_fast_kernel"],
               "c3": ["bpe_lane_kernel", "bpe_fast_kernel", "bpe_compact_kernel"],
               "ja": ["unigram_fast_kernel<16, false, 3"],
               "ja_coop": ["coop_list_kernel"],
               "c4": ["estep_backward_kernel"],
               # (the PARITY forward pass is the encode byte kernel's E-step mode)
               "c4_pipeline": ["unigram_fast_kernel<16, true, 4, true", "estep_backward_kernel",
                               "estep_compact_records_kernel", "estep_fold_kernel"]}


def encode_leg(args, model_path, steps, warmup, world, rank, dev, dist, pmc_leg, probe_stats, corpus=None,
               workload=None, period=None, coop=False):
    """One encode benchmark (c2 unigram or c3 BPE on synthetic text, or a
    given normalized `corpus` (buf, off) described by `workload`) on this
    rank's shard."""
    import numpy as np
    import torch
    import spm_amd
    import synth
    model_bytes = open(model_path, "rb").read()
    torch.cuda.reset_peak_memory_stats(dev)
    spm_amd.device_peak_reset()
    dm = spm_amd.DeviceModel(model_bytes)
    dm.set_timing(True)
    info = dm.info()
    t0 = time.time()
    buf, off = corpus if corpus is not None else synth.normalized(args.sentences, seed=1234 + rank)
    gen_s = time.time() - t0
    n = len(off) - 1
    total_bytes = int(off[-1])
    d_bytes = torch.from_numpy(buf).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_ids = torch.empty(max(total_bytes, 1), dtype=torch.int32, device=dev)
    d_tok = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_st = torch.zeros(1, dtype=torch.int32, device=dev)
    sp = torch.cuda.current_stream(dev).cuda_stream

    def step():
        # The pure stream call: no host synchronization inside a step.
        dm.encode_device_async(d_bytes.data_ptr(), d_off.data_ptr(), n, total_bytes, d_ids.data_ptr(),
                               d_tok.data_ptr(), d_st.data_ptr(), stream=sp)

    for _ in range(max(warmup, 1)):  # at least one untimed call: the token count to compare against
        step()
    torch.cuda.synchronize(dev)
    if int(d_st.item()) != 0:
        raise RuntimeError("encode status %d" % int(d_st.item()))
    ntok = int(d_tok[-1].item())
    dm.drain_kernel_times(sp)  # drop the warm-up launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # Fast-kernel HIP events of the K timed launches (on the encode stream).
    fast_ms = dm.drain_kernel_times(sp)
    if int(d_st.item()) != 0 or int(d_tok[-1].item()) != ntok:
        raise RuntimeError("encode status %d / token count changed" % int(d_st.item()))
    check = None
    if rank == 0 and not args.no_parity_check:
        ids_t = d_ids[:ntok].cpu().numpy()
        to_t = d_tok.cpu().numpy()
    # General-path count (and the piece byte lengths for the parity check)
    # from one blocking call outside the timed region.
    d_len = torch.empty(max(total_bytes, 1), dtype=torch.int32, device=dev) if rank == 0 else None
    dm.encode_device(d_bytes.data_ptr(), d_off.data_ptr(), n, d_ids.data_ptr(), d_tok.data_ptr(),
                     d_len=d_len.data_ptr() if d_len is not None else None, stream=sp)
    st = dm.stats()
    general, gen_ms = st.general_path, [st.general_kernel_ms]
    if rank == 0 and not args.no_parity_check:
        torch.cuda.synchronize(dev)
        again = (np.array_equal(d_ids[:ntok].cpu().numpy(), ids_t) and
                 np.array_equal(d_tok.cpu().numpy(), to_t))
        lens = d_len[:ntok].cpu().numpy().view(np.uint32)
        log("full-size parity check (%s)" % os.path.basename(model_path))
        check = parity_encode(model_bytes, buf, off, ids_t, lens, to_t.view(np.uint64),
                              min(args.cpu_threads, os.cpu_count() or 1), period)
        check["blocking_call_equal_to_timed"] = bool(again)
        if not again:
            check["mismatches"] += 1
    del d_len
    # Per-sentence token counts (rank 0), for the cooperative path's share of
    # the algorithmic bytes below.
    tok_counts = np.diff(d_tok.cpu().numpy().view(np.uint64)) if (rank == 0 and coop) else None
    total_sent = float(n)
    # Device bytes per rank at the high-water mark: the library's own blocks
    # (model, encode workspace; spm_hip_device_bytes) and torch's (the
    # resident corpus, offsets, ids and token offsets).
    mem = [float(spm_amd.device_bytes()[1]), float(torch.cuda.max_memory_allocated(dev))]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([float(n)], dtype=torch.float64, device=dev)
        dist.all_reduce(tot)
        total_sent = float(tot.item())
        mt = torch.tensor(mem, dtype=torch.float64, device=dev)
        dist.all_reduce(mt, op=dist.ReduceOp.MAX)
        mem = mt.tolist()
    del d_bytes, d_off, d_ids, d_tok
    torch.cuda.empty_cache()
    if rank != 0:
        return None, model_bytes
    unigram = info.model_type == spm_amd.SPM_UNIGRAM
    # Algorithmic bytes of one launch: normalized bytes +
    # offsets (8 B) read, ids (4 B/token) + token offsets (8 B) written.
    algo_bytes = total_bytes + 8 * (n + 1) + 4 * ntok + 8 * (n + 1)
    k_ms = float(np.mean(fast_ms))
    kname = kernel_label(info, spm_amd)
    achieved = algo_bytes / (k_ms * 1e-3) / 1e9
    traffic, tinfo = pmc_traffic(args.pmc_dir, pmc_leg, PMC_KERNELS[pmc_leg])
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": kname, "kernel_ms": k_ms, "algo_bytes_per_launch": algo_bytes,
            "general_kernel_ms": float(np.mean(gen_ms))}
    roof.update(tinfo)
    if coop and tok_counts is not None:
        # Long lines take the cooperative kernel (one sentence per wave,
        # nb >= the model's coop threshold); on real text
        # it dominates the step, so it gets its own roofline: its sentences'
        # algorithmic bytes over the path's event time (coop_list_kernel +
        # unigram_general_kernel, one blocking call), PMC traffic of
        # coop_list_kernel from its committed summary.
        lens = (off[1:] - off[:-1]).astype(np.uint64)
        sel = lens >= COOP_MIN_NB
        c_algo = int(lens[sel].sum()) + 16 * int(sel.sum()) + 4 * int(tok_counts[sel].sum())
        c_ms = float(np.mean(gen_ms))
        c_ach = c_algo / (c_ms * 1e-3) / 1e9 if c_ms > 0 else 0.0
        c_traffic, c_info = pmc_traffic(args.pmc_dir, "ja_coop", PMC_KERNELS["ja_coop"])
        roof["coop"] = {"bound": "hbm", "kernel": "coop_list_kernel (+ unigram_general_kernel)", "kernel_ms": c_ms,
                        "sentences_per_launch": int(sel.sum()), "algo_bytes_per_launch": c_algo,
                        "achieved": c_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": c_ach / HBM_PEAK_GBS,
                        "traffic": c_traffic, "coop_rest": int(st.coop_rest)}
        roof["coop"].update(c_info)
    if unigram and probe_stats:
        ts = dm.trie_stats(buf, off, BOX_CPU_SHARE)
        s = k_ms * 1e-3
        roof.update({"trie_char_starts_per_launch": ts.char_starts,
                     "trie_unit_loads_per_launch": ts.unit_loads,
                     "trie_leaf_loads_per_launch": ts.leaf_loads,
                     "trie_unit_loads_per_s": ts.unit_loads / s,
                     "trie_probes_per_s": (ts.unit_loads + ts.leaf_loads) / s,
                     "trie_probe_note": "unit loads = dependent double-array steps of every char-start walk "
                                        "(mismatching probe included); leaf loads = one score load per "
                                        "matched piece (spm_hip_model_trie_stats, host count)"})
    ms_per_step = elapsed * 1000.0 / steps
    line = {
        "metric": ("sentences/sec Encode (32k unigram) @%d GPU" if unigram
                   else "sentences/sec Encode (32k BPE) @%d GPU") % world,
        "value": total_sent * steps / elapsed,
        "unit": "sentences/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/f32",
        "data": "synthetic",
        "config": {"workload": (workload or (("c2: batched unigram Viterbi Encode" if unigram else
                                              "c3: BPE Encode merge loop") +
                                             ", %d synthetic normalized sentences/GPU" % n)) +
                               " (mean %.2f B), model %s" % (total_bytes / max(n, 1),
                                                              os.path.relpath(model_path, ROOT)),
                   "sentences_per_gpu": n, "tokens_per_gpu": ntok,
                   "general_path_sentences": int(general),
                   "parallelism": "dp%d (sharded corpus, no collective)" % world},
        "roofline": roof,
        "synth_gen_s": gen_s,
        "peak_device_bytes_per_rank": {"library": int(mem[0]), "torch_buffers": int(mem[1]),
                                       "total": int(mem[0] + mem[1]), "reduction": "max over ranks"},
    }
    if check is not None:
        line["parity_check"] = check
    return line, model_bytes


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0 and args.gpus > 1:
        sys.exit(launch_workers(args))
    world = max(world, 1)
    import torch
    import torch.distributed as dist
    if args.dry_run:
        return dry_run(args, world, torch, dist)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    log("c2 encode leg")
    line, model_bytes = encode_leg(args, args.model, args.steps, args.warmup, world, rank, dev, dist,
                                   "c2", not args.no_probe_stats)
    if rank == 0 and not args.no_cpu_baseline:
        log("c2 cpu baseline")
        th = min(args.cpu_threads, os.cpu_count() or 1)
        cb = cpu_encode_baseline(model_bytes, args.cpu_sample, th)
        one = cpu_encode_baseline(model_bytes, args.cpu_sample_1t, 1)
        cb["single_thread"] = one
        cb["note"] = ("oracle restatement, not the reference build (unbuildable here, DESIGN.md §2); "
                      "SURVEY §6 measured the reference at 523k sentences/s with 8 threads")
        line["cpu_baseline"] = cb
    if args.bpe_steps > 0 and os.path.exists(args.bpe_model):
        log("c3 BPE leg")
        bl, bpe_bytes = encode_leg(args, args.bpe_model, args.bpe_steps, min(args.warmup, 2), world, rank, dev,
                                   dist, "c3", False)
        if rank == 0:
            if not args.no_cpu_baseline:
                log("c3 cpu baseline")
                bl["cpu_baseline"] = cpu_encode_baseline(bpe_bytes, args.cpu_sample // 4,
                                                         min(args.cpu_threads, os.cpu_count() or 1))
            line["bpe_c3"] = bl
    if args.ja_lines > 0:
        log("multi-byte (ja) leg")
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        ja = multibyte_leg(args, world, rank, dev, dist)
        if rank == 0:
            line["ja_multibyte"] = ja
    if args.raw_steps > 0:
        log("raw e2e leg")
        e2e = raw_e2e_bench(args, world, rank, dev, dist)
        if rank == 0:
            line["e2e_raw"] = e2e
    if args.estep_sentences > 0:
        log("c4 E-step leg")
        es = estep_bench(args, model_bytes, world, rank, dev, dist)
        if rank == 0:
            line["estep"] = es
    # Hand this process's cached device memory back before the trainer
    # children allocate theirs.
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and args.latency_calls > 0:
        log("latency leg")
        line["latency"] = latency_bench(args)
    if rank == 0 and world == 1 and args.train_lines > 0:
        log("c5 train leg")
        line["train"] = train_bench(args)
    if rank == 0 and world == 1 and args.bpe_train_lines > 0:
        log("BPE train leg")
        line["train_bpe"] = bpe_train_bench(args)
    bad = 0
    if rank == 0 and not args.no_parity_check:
        # Full-size parity of the benchmarked workloads: every
        # checked leg must be bit-exact; any mismatch fails the bench.
        par = {}
        if "parity_check" in line:
            par["c2"] = line.pop("parity_check")
        if "parity_check" in line.get("bpe_c3", {}):
            par["c3"] = line["bpe_c3"].pop("parity_check")
        if "parity_check" in line.get("ja_multibyte", {}):
            par["ja_multibyte"] = line["ja_multibyte"].pop("parity_check")
        if "check" in line.get("estep", {}):
            par["c4_parity"] = line["estep"].pop("check")
        if "cpu_baseline" in line.get("train", {}):
            par["c5_sample"] = {"mismatches": 0 if line["train"]["cpu_baseline"]["piece_table_bit_identical"] else 1,
                                "compared": "piece table of lib/spm_train vs the oracle trainer on the "
                                            "%d-line sample" % args.train_cpu_sample}
        bad = sum(int(v["mismatches"]) for v in par.values())
        par["mismatches_total"] = bad
        line["parity"] = par
    if rank == 0:
        try:
            os.makedirs(os.path.dirname(args.detail), exist_ok=True)
            with open(args.detail, "w") as f:
                json.dump(line, f, indent=1)
        except OSError as e:
            log("detail file not written: %s" % e)
        print(json.dumps(compact_line(line, os.path.relpath(args.detail, ROOT))), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if bad:
        raise ParityError("full-size parity check: %d mismatches (see the line's parity object)" % bad)


ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms", "algo_bytes_per_launch",
             "traffic_stamp", "traffic_note", "traffic_per_sentence", "pipeline_traffic_per_sentence", "coop_rest")


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _roof(r):
    if not isinstance(r, dict):
        return r
    out = _pick(r, ROOF_KEYS)
    if "coop" in r:
        out["coop"] = _pick(r["coop"], ROOF_KEYS)
    return out


def compact_line(full, detail_path):
    """The printed line: the contract keys and every leg's numbers (about
    5 KB, so the driver's output tail holds all of it), ending with `legs`:
    value, roofline frac and PMC traffic per leg.  The full record (notes,
    logs, per-batch tables, stage dicts) is in the detail side file."""
    head = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")
    line = _pick(full, head)
    line["roofline"] = _roof(full.get("roofline"))
    if "cpu_baseline" in full:
        cb = full["cpu_baseline"]
        line["cpu_baseline"] = _pick(cb, ("value", "unit", "cores", "kind", "sample"))
        if "single_thread" in cb:
            line["cpu_baseline"]["single_thread_value"] = cb["single_thread"]["value"]
    line["peak_device_bytes_per_rank"] = full.get("peak_device_bytes_per_rank", {}).get("total")
    legs = {"c2": {"value": full.get("value"), "unit": full.get("unit"),
                   "frac": (full.get("roofline") or {}).get("frac"),
                   "traffic": (full.get("roofline") or {}).get("traffic")}}
    for key, name in (("bpe_c3", "c3"), ("ja_multibyte", "ja")):
        leg = full.get(key)
        if not leg:
            continue
        line[key] = _pick(leg, ("metric", "value", "unit", "ms_per_step"))
        line[key]["roofline"] = _roof(leg.get("roofline"))
        line[key]["general_path_sentences"] = leg.get("config", {}).get("general_path_sentences")
        line[key]["peak_device_bytes"] = leg.get("peak_device_bytes_per_rank", {}).get("total")
        if "cpu_baseline" in leg:
            line[key]["cpu_baseline"] = _pick(leg["cpu_baseline"], ("value", "unit", "cores", "kind"))
        r = leg.get("roofline") or {}
        legs[name] = {"value": leg.get("value"), "unit": leg.get("unit"), "frac": r.get("frac"),
                      "traffic": r.get("traffic")}
        if "coop" in r:
            legs["ja_coop"] = {"frac": r["coop"].get("frac"), "traffic": r["coop"].get("traffic"),
                               "kernel_ms": r["coop"].get("kernel_ms")}
    if full.get("e2e_raw"):
        line["e2e_raw"] = _pick(full["e2e_raw"], ("metric", "value", "unit", "ms_per_step", "gpu_ms_per_step"))
        legs["e2e_raw"] = {"value": full["e2e_raw"].get("value"), "unit": "sentences/s"}
    es = full.get("estep")
    if es:
        line["estep"] = _pick(es, ("metric", "value", "unit", "higher_is_better", "n_gpus", "sentences_per_epoch",
                                   "sentences_per_s", "mode", "collective", "repeat_epoch_bit_identical"))
        line["estep"]["roofline"] = _roof(es.get("roofline"))
        if "cpu_baseline" in es:
            line["estep"]["cpu_baseline"] = _pick(es["cpu_baseline"], ("value", "unit", "cores", "kind"))
        r = es.get("roofline") or {}
        legs["c4"] = {"value": es.get("value"), "unit": "s/epoch", "frac": r.get("frac"), "traffic": r.get("traffic")}
    lat = full.get("latency")
    if lat:
        b1 = [b["us_per_call"] for b in lat.get("batches", []) if b["batch"] == 1]
        c1 = lat.get("c1_botchan", {})
        line["latency"] = {"encode_line_us": lat.get("encode_single_us"), "batch1_us": b1[0] if b1 else None,
                           "crossover_batch": lat.get("crossover_batch"),
                           "c1_line_by_line_sentences_per_s": c1.get("line_by_line_sentences_per_s"),
                           "c1_reference_sentences_per_s": c1.get("reference_sentences_per_s"),
                           "c1_file_sentences_per_s": c1.get("file_sentences_per_s")}
        legs["c1_line"] = {"value": c1.get("line_by_line_sentences_per_s"), "unit": "sentences/s"}
    tr = full.get("train")
    if tr:
        line["train"] = _pick(tr, ("metric", "value", "unit", "lines", "peak_device_bytes"))
        line["train"]["stage_s"] = {k: v for k, v in tr.get("stages", {}).items()
                                    if k in ("load_s", "seed_s", "split_s", "estep_s", "mstep_s", "prune_s",
                                             "finalize_s")}
        line["train"]["stage_peak_bytes"] = tr.get("stages", {}).get("stage_peak_bytes")
        if "cpu_baseline" in tr:
            line["train"]["cpu_baseline"] = _pick(tr["cpu_baseline"], ("value", "unit", "cores", "kind",
                                                                       "gpu_same_sample_s"))
        legs["c5"] = {"value": tr.get("value"), "unit": "s"}
    tb = full.get("train_bpe")
    if tb:
        st = tb.get("stages", {})
        line["train_bpe"] = _pick(tb, ("metric", "value", "unit", "lines", "merge_loop_s"))
        line["train_bpe"]["stage_s"] = {k: v for k, v in st.items()
                                        if k.startswith("bpe_") and k.endswith("_s")}
        legs["bpe_train"] = {"value": tb.get("value"), "unit": "s", "bpe_update_s": st.get("bpe_update_s")}
    if "parity" in full:
        line["parity"] = {k: (v.get("mismatches") if isinstance(v, dict) else v) for k, v in full["parity"].items()}
    line["detail"] = detail_path
    line["legs"] = legs
    return line


def dry_run(args, world, torch, dist):
    """Launcher/rendezvous check without a GPU (gloo): every rank reports its
    shard size; rank 0 prints the summed count and the max-over-ranks time."""
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    tot = torch.tensor([float(args.sentences)], dtype=torch.float64)
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tot)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "dry-run (launcher check, no GPU work)", "value": float(tot.item()),
                          "unit": "sentences", "n_gpus": world, "steps": 0, "warmup": 0,
                          "ms_per_step": float(el.item()) * 1000.0, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "u8/f32", "data": "none",
                          "config": {"workload": "dry-run", "parallelism": "dp%d" % world}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _train_run(args, lines, model_type, extra=""):
    """One lib/spm_train run through tools/train_bench.py in a child process
    (the child draws the synthetic corpus with a process pool and has never
    touched the GPU; spm_train is its own child).  Returns the --timings JSON
    plus corpus generation time and sizes."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "train_bench.py"), "--lines", str(lines),
           "--workers", str(BOX_CPU_SHARE), "--model-type", model_type,
           "--args", "--normalization_rule_name=identity --num_threads=16" + extra]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    if p.returncode != 0:
        raise RuntimeError(p.stderr.decode(errors="replace")[-2000:])
    return json.loads(p.stdout.decode().strip().splitlines()[-1])


def train_bench(args):
    """c5: full `spm_train --model_type=unigram --vocab_size=32000` (lib/spm_train:
    device seed mining, device E-steps in PARITY mode with 16 buckets, device
    pruning Viterbi) on BASELINE config 5's 100M synthetic lines.  One run =
    the whole training, file read to .model/.vocab written (corpus drawing
    excluded).  The CPU baseline is the oracle trainer
    (oracle/spm_oracle_train.inc, single-thread seed mining, 16-bucket
    threaded E-step) on a bounded sample, with the GPU trainer run on the
    same sample beside it; the two .model files must be byte-identical
    (parity check, not only timing).  The reference cannot run 100M lines at
    all (int32 esaxx, unigram_model_trainer.cc:150-164)."""
    import tempfile
    import train_bench as tb
    spec = "--normalization_rule_name=identity --num_threads=16"
    log("c5: %d lines" % args.train_lines)
    tm = _train_run(args, args.train_lines, "unigram")
    res = {"metric": "spm_train unigram 32k end-to-end @1 GPU", "value": tm["total_s"], "unit": "s",
           "higher_is_better": False, "lines": args.train_lines, "stages": tm,
           "peak_device_bytes": tm.get("peak_device_bytes"),
           "stage_peak_device_bytes": dict(zip(("load", "seed", "split", "em_prune_finalize"),
                                               tm.get("stage_peak_bytes", []))),
           "workload": "c5: spm_train --model_type=unigram --vocab_size=32000 %s on %d synthetic "
                       "lines (tools/synth.py raw text, %.2f GB), file read to .model written"
                       % (spec, args.train_lines, tm["corpus_bytes"] / 1e9)}
    d = tempfile.mkdtemp(prefix="spm_c5_")
    if not args.no_cpu_baseline and args.train_cpu_sample > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        corpus = os.path.join(d, "sample.txt")
        tb.write_corpus(corpus, args.train_cpu_sample, 1234)
        cmd = [tb.TRAIN, "--input=" + corpus, "--model_prefix=" + os.path.join(d, "sample"),
               "--model_type=unigram", "--vocab_size=32000", "--timings"] + spec.split()
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        if p.returncode != 0:
            raise RuntimeError(p.stderr.decode(errors="replace")[-2000:])
        gtm = json.loads(p.stdout.decode().strip().splitlines()[-1])
        log("c5 oracle trainer on the sample")
        lines = oracle_lib.read_lines_binary(corpus)
        t0 = time.perf_counter()
        ot = oracle_lib.OracleTrainer("--vocab_size=32000 " + spec, lines)
        wp, ws, wt = ot.train()
        dt = time.perf_counter() - t0
        import numpy as np
        import model_reader
        got = model_reader.read_pieces(open(os.path.join(d, "sample.model"), "rb").read())
        parity = ([g[0] for g in got] == list(wp) and [g[2] for g in got] == list(wt) and
                  np.array_equal(np.array([g[1] for g in got], dtype=np.float32).view(np.uint32),
                                 np.asarray(ws, dtype=np.float32).view(np.uint32)))
        if not parity:
            raise RuntimeError("c5 sample: lib/spm_train piece table differs from the oracle trainer's")
        res["cpu_baseline"] = {"value": dt, "unit": "s", "cores": 16, "kind": "port",
                               "sample": "%d lines of the same generator; oracle trainer (single-thread "
                                         "load/seed/prune, 16-bucket threaded E-step) %.1f s vs "
                                         "lib/spm_train %.2f s on the same sample"
                                         % (args.train_cpu_sample, dt, gtm["total_s"]),
                               "gpu_same_sample_s": gtm["total_s"],
                               "piece_table_bit_identical": parity}
    return res


COOP_MIN_NB = 128  # spm_hip_api.cc DefaultCoopMinNb(): sentences of >= 128 bytes take the cooperative kernel
REF_US_PER_SENTENCE = 1e6 / 108.5e3  # reference Encode, 1 thread, ~25-char sentences


def multibyte_leg(args, world, rank, dev, dist):
    """Real multi-byte text: the reference's test_ja_model.model on its own
    wagahaiwa_nekodearu.txt (both in tests/golden/), the 2344 lines repeated
    to >= --ja-lines lines, normalized by the model's own rules on the host,
    then timed like c2 (normalized bytes resident in HBM).  Reports the
    kernel the model selects and how many sentences take the general path."""
    import numpy as np
    import oracle_lib
    import spm_amd
    gold = os.path.join(ROOT, "tests", "golden")
    mpath = os.path.join(gold, "test_ja_model.model")
    lines = [l for l in oracle_lib.read_lines_binary(os.path.join(gold, "wagahaiwa_nekodearu.txt"))]
    reps = (args.ja_lines + len(lines) - 1) // len(lines)
    dm = spm_amd.DeviceModel(open(mpath, "rb").read(), host_only=True)  # host normalizer only
    rb, ro = spm_amd.to_csr(lines)
    nb, no = dm.normalize_csr(rb, ro, threads=BOX_CPU_SHARE)
    dm.close()
    base = len(no) - 1
    ln = (no[1:] - no[:-1]).astype(np.uint64)
    lens = np.tile(ln, reps)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens, dtype=np.uint64)
    buf = np.tile(nb[:int(no[-1])], reps)
    line, _ = encode_leg(args, mpath, args.steps, args.warmup, world, rank, dev, dist, "ja", False,
                         corpus=(buf, off), period=base, coop=True,
                         workload="real multi-byte text: tests/golden/wagahaiwa_nekodearu.txt (%d lines) x %d = %d "
                                  "sentences normalized by test_ja_model.model's rules" % (base, reps, len(lens)))
    return line


def latency_bench(args):
    """The plugin point's per-call latency (lib/spm_latency, a child process):
    SentencePieceProcessor::Encode(line, &ids) one line per call, and
    spm_hip_encode_batch_host over B normalized sentences for B = 1..65536;
    `crossover_batch` = the smallest B whose per-sentence cost beats the
    reference's single-core 9.2 us."""
    import tempfile
    import synth
    d = tempfile.mkdtemp(prefix="spm_lat_")
    path = os.path.join(d, "lines.txt")
    with open(path, "wb") as f:
        f.write(b"\n".join(synth.lines(70000, seed=77)) + b"\n")
    exe = os.path.join(ROOT, "sentencepiece-comments_amd", "lib", "spm_latency")
    p = subprocess.run([exe, args.model, path, str(args.latency_calls)], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE)
    if p.returncode != 0:
        raise RuntimeError(p.stderr.decode(errors="replace")[-2000:])
    res = json.loads(p.stdout.decode().strip().splitlines()[-1])
    cross = [b["batch"] for b in res["batches"] if b["us_per_sentence"] < REF_US_PER_SENTENCE]
    res["reference_us_per_sentence"] = REF_US_PER_SENTENCE
    res["crossover_batch"] = cross[0] if cross else None
    res["workload"] = ("synthetic raw lines (tools/synth.py seed 77), model %s; Encode(single) = raw line -> "
                       "device normalize + encode + id epilogue -> host ids" % os.path.relpath(args.model, ROOT))
    # c1: botchan with test_model.model (BASELINE config 1), the whole file as
    # one EncodeBatch(ids) call and line by line; reference 28.3k sent/s (1 thread).
    gold = os.path.join(ROOT, "tests", "golden")
    p = subprocess.run([exe, os.path.join(gold, "test_model.model"), os.path.join(gold, "botchan.txt"), "4288"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    if p.returncode != 0:
        raise RuntimeError(p.stderr.decode(errors="replace")[-2000:])
    c1 = json.loads(p.stdout.decode().strip().splitlines()[-1])
    res["c1_botchan"] = {"file_sentences_per_s": c1["encode_file_sentences_per_s"], "file_s": c1["encode_file_s"],
                         "line_by_line_sentences_per_s": 1e6 / c1["encode_single_us"],
                         "encode_single_us": c1["encode_single_us"], "lines": c1["lines"],
                         "reference_sentences_per_s": 28.3e3,
                         "workload": "c1: tests/golden/botchan.txt (4288 lines) + test_model.model, raw lines -> ids "
                                     "(device normalize + encode + id epilogue), one EncodeBatch call for the file "
                                     "and one Encode call per line"}
    return res


def bpe_train_bench(args):
    """BPE trainer (bpe_model_trainer.cc:185-330) on --bpe-train-lines
    synthetic lines, vocab 32000: device pair census + host merge loop, with
    the merge loop's stage breakdown (trainer --timings)."""
    tm = _train_run(args, args.bpe_train_lines, "bpe")
    return {"metric": "spm_train bpe 32k end-to-end @1 GPU", "value": tm["total_s"], "unit": "s",
            "higher_is_better": False, "lines": args.bpe_train_lines, "stages": tm,
            "merge_loop_s": tm["estep_s"],
            "workload": "spm_train --model_type=bpe --vocab_size=32000 on %d synthetic lines" % args.bpe_train_lines}


def raw_e2e_bench(args, world, rank, dev, dist):
    """Raw text → ids on the device: the c2 corpus size as RAW lines resident
    in HBM, split into two batches that are pipelined on one stream with the
    pure stream calls (no host synchronization in a step): per batch
    spm_hip_normalize_batch_device_async (Normalizer::Normalize with the
    model's nmt_nfkc charsmap: length pass, scan, write pass) +
    spm_hip_encode_batch_async + spm_hip_finalize_ids_async (the unk-run
    merge of PopulateSentencePieceText), i.e. SentencePieceProcessor::
    Encode(ids) per line; one status word per batch.  Weak-scaled like c2."""
    import numpy as np
    import torch
    import spm_amd
    import synth
    dm = spm_amd.DeviceModel(open(args.model, "rb").read())
    sp = torch.cuda.current_stream(dev).cuda_stream
    batches = []
    half = args.sentences // 2
    for k, cnt in enumerate((half, args.sentences - half)):
        buf, off = synth.raw(cnt, seed=1234 + rank + 7919 * k)
        cap = int(off[-1]) * 2 + 4 * cnt  # > normalized size (checked by the status word)
        bt = {"n": cnt, "raw": int(off[-1]), "cap": cap,
              "in": torch.from_numpy(buf).to(dev), "in_off": torch.from_numpy(off.view(np.int64)).to(dev),
              "norm": torch.empty(cap, dtype=torch.uint8, device=dev),
              "noff": torch.empty(cnt + 1, dtype=torch.int64, device=dev),
              "ids": torch.empty(cap, dtype=torch.int32, device=dev),
              "tok": torch.empty(cnt + 1, dtype=torch.int64, device=dev),
              "fin": torch.empty(cap, dtype=torch.int32, device=dev),
              "fin_off": torch.empty(cnt + 1, dtype=torch.int64, device=dev),
              "st": torch.zeros(1, dtype=torch.int32, device=dev)}
        batches.append(bt)
    n = sum(bt["n"] for bt in batches)

    def chain(bt):
        dm.normalize_device_async(bt["in"].data_ptr(), bt["in_off"].data_ptr(), bt["n"], bt["norm"].data_ptr(),
                                  bt["cap"], bt["noff"].data_ptr(), bt["st"].data_ptr(), stream=sp)
        dm.encode_device_async(bt["norm"].data_ptr(), bt["noff"].data_ptr(), bt["n"], bt["cap"],
                               bt["ids"].data_ptr(), bt["tok"].data_ptr(), bt["st"].data_ptr(), stream=sp)
        dm.finalize_ids_device_async("", bt["ids"].data_ptr(), bt["tok"].data_ptr(), bt["n"], bt["fin"].data_ptr(),
                                     bt["cap"], bt["fin_off"].data_ptr(), bt["st"].data_ptr(), stream=sp)

    def step():
        for bt in batches:
            chain(bt)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.raw_steps):
        step()
    ev1.record()
    host_enqueue_s = time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1) / args.raw_steps
    codes = [int(bt["st"].item()) for bt in batches]
    if any(codes):
        raise RuntimeError("raw chain status %r" % codes)
    norm_bytes = sum(int(bt["noff"][-1].item()) for bt in batches)
    raw_bytes = sum(bt["raw"] for bt in batches)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    dm.close()
    return {"metric": "sentences/sec raw text -> ids (device Normalize + Encode + id epilogue) @%d GPU" % world,
            "value": n * world * args.raw_steps / el, "unit": "sentences/s", "steps": args.raw_steps,
            "ms_per_step": el * 1000.0 / args.raw_steps, "gpu_ms_per_step": gpu_ms,
            "host_enqueue_ms_per_step": host_enqueue_s * 1000.0 / args.raw_steps,
            "batches_per_step": len(batches), "raw_bytes_per_gpu": raw_bytes,
            "normalized_bytes_per_gpu": norm_bytes,
            "workload": "%d raw synthetic lines/GPU resident in HBM (mean %.2f B) in 2 batches pipelined on one "
                        "stream with the *_async calls (zero host synchronizations per step), model %s (nmt_nfkc)"
                        % (n, raw_bytes / max(n, 1), os.path.relpath(args.model, ROOT))}


def estep_bench(args, model_bytes, world, rank, dev, dist):
    """c4: unigram trainer E-step over a fixed corpus (default 100M synthetic
    normalized sentences, freq 1, no whitespace split) sharded over the ranks
    (strong scaling), pieces = the NORMAL pieces of the 32k model.

    PARITY (the mode spm_train ships): T = --estep-threads ordered float
    buckets (sentence i → bucket i mod T, the reference's thread), bit-exact
    to RunEStep at num_threads = T; rank r owns the buckets b ≡ r (mod
    world); at world > 1 one all-gather of the owned float[V] rows (+ SUM of
    obj / ntok).  (The fp64 FAST mode is no faster and is not benchmarked.)"""
    import numpy as np
    import torch
    import dist_estep
    import spm_amd
    import synth
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import model_reader
    pcs = [(p, s) for p, s, t in model_reader.read_pieces(model_bytes) if t == 1]
    pieces = [p for p, _ in pcs]
    scores = np.array([s for _, s in pcs], dtype=np.float32)
    dp = spm_amd.DevicePieces(pieces, scores)
    total = args.estep_sentences
    m = min(args.estep_buffer, total)
    buf, off = synth.normalized(m, seed=99 + rank)
    d_b = torch.from_numpy(buf).to(dev)
    d_o = torch.from_numpy(off.view(np.int64)).to(dev)
    d_f = torch.ones(m, dtype=torch.int64, device=dev)
    ar = (lambda x: dist.all_reduce(x)) if world > 1 else None

    def ag(x):  # PARITY: every rank's packed owned rows (dist_estep.gather_owned_rows)
        out = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(out, x)
        return out

    def clock():
        torch.cuda.synchronize(dev)
        return time.perf_counter()

    def timed(mode, T, chunks, epochs, warm):
        runner = dist_estep.DeviceEStep(dp, mode, T, dev, total)
        times = {}
        kt = {}

        epoch = dist_estep.make_epoch(chunks, mode, T, dp.V, runner.accumulate, runner.finalize, runner.make_zeros,
                                      world=world, rank=rank, all_reduce=ar, all_gather=ag, sync=runner.sync,
                                      clock=clock)

        for _ in range(warm):
            epoch()
            log("E-step mode %d warm-up epoch done" % mode)
        torch.cuda.synchronize(dev)
        dp.set_timing(True)
        dp.kernel_times()  # (reset)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(epochs):
            e, o, nt = epoch()
            log("E-step mode %d epoch done" % mode)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        # Forward / backward pass durations of the timed epochs (HIP events on
        # the E-step's stream around every chunk's launches).
        fwd_ms, bwd_ms, nchunks = dp.kernel_times()
        dp.set_timing(False)
        kt.update({"forward_ms": fwd_ms, "backward_ms": bwd_ms, "chunks": nchunks})
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        # One more epoch, outside the timed region, with a device sync between
        # this rank's accumulate calls and the collectives: where an epoch's
        # time goes per rank (compute vs exchange), for the scaling runs.
        e2, o2, nt2 = epoch(times)
        split = {"compute_s": times["compute_s"], "collective_s": times["collective_s"], "path": times["path"]}
        if world > 1:
            t = torch.tensor([split["compute_s"], split["collective_s"]], dtype=torch.float64, device=dev)
            allt = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(allt, t)
            split["per_rank_compute_s"] = [float(x[0].item()) for x in allt]
            split["per_rank_collective_s"] = [float(x[1].item()) for x in allt]
        same = bool(torch.equal(e, e2)) and float(o.item()) == float(o2.item()) and int(nt.item()) == int(nt2.item())
        split["kernel_times"] = kt
        return el / epochs, int(nt.item()), float(o.item()), e, split, same

    # Roofline of the dominant kernel (the backward pass), SURVEY §8d c4:
    # algorithmic bytes per sentence = normalized text + 8 (offset) + 8 (freq);
    # one launch = one accumulate chunk of this rank's sentences.
    norm_mean = float(off[-1]) / m
    algo_ps = norm_mean + 16.0

    def roof(split, sec_epoch, epochs, rank_sentences, kname):
        kt = split.get("kernel_times") or {}
        nch = kt.get("chunks", 0)
        if not nch:
            return None
        per_chunk = rank_sentences * epochs / nch
        bwd = kt["backward_ms"] / nch
        algo = algo_ps * per_chunk
        ach = algo / (bwd / 1e3) / 1e9
        return {"bound": "hbm", "kernel": kname, "algo_bytes_per_sentence": algo_ps,
                "algo_bytes_per_launch": algo, "sentences_per_launch": per_chunk, "kernel_ms": bwd,
                "forward_kernel_ms": kt["forward_ms"] / nch, "launches_timed": nch,
                "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                "traffic": None, "epoch_algo_gbs": algo_ps * total / sec_epoch / 1e9}

    T = args.estep_threads
    coll = ("one RCCL all-gather of each rank's owned float[V] bucket rows + SUM all-reduce of obj[T] / "
            "ntok[T] per epoch" if world > 1 else "single GPU, no collective")
    res = {"metric": "E-step sec/epoch @%d GPU" % world, "unit": "s/epoch", "higher_is_better": False,
           "n_gpus": world, "sentences_per_epoch": total, "pieces": dp.V,
           "mode": "PARITY (T=%d ordered float buckets, bit-exact to RunEStep at num_threads=%d)" % (T, T),
           "collective": coll,
           "workload": "c4: %d synthetic normalized sentences/epoch (freq 1, no whitespace split, mean %.2f "
                       "normalized B), NORMAL pieces of data/synth32k_unigram.model, sharded over %d rank(s) by "
                       "bucket ownership" % (total, norm_mean, world)}
    # PARITY, the mode spm_train ships: this rank's whole buckets, interleaved
    # in sentence order (the shard plan spm_train --num_gpus uses,
    # csrc/shard_plan.h): every call holds all of the rank's buckets, so their
    # float chains fold in parallel.
    pchunks = []
    for base, stride, cnt in spm_amd.estep_shard_plan(total, dist_estep.PARITY, T, world, rank):
        done = 0
        while done < cnt:
            k = min(cnt - done, m)
            pchunks.append({"b": d_b, "o": d_o, "f": d_f, "n": k, "base": base + stride * done,
                            "stride": stride})
            done += k
    w0, k0 = dp.record_stats()
    psec, pnt, pob, pe, psplit, prepeat = timed(dist_estep.PARITY, T, pchunks, args.estep_parity_epochs,
                                                args.estep_warmup)
    w1, k1 = dp.record_stats()
    rank_sent = sum(c["n"] for c in pchunks)
    rl = roof(psplit, psec, args.estep_parity_epochs, rank_sent, "estep_backward_kernel<16, 4, 42> (PARITY)")
    if rl is not None:
        # PMC bytes per sentence of the profiled steady (record-drop)
        # dispatches, scaled to this run's sentences per launch; and the whole
        # per-chunk pipeline's bytes per sentence (forward, backward, record
        # compaction, fold).
        import pmc_stamp
        per_ps = {}
        for kern in PMC_KERNELS["c4_pipeline"]:
            b, info = pmc_traffic(args.pmc_dir, "c4", [kern])
            path = os.path.join(args.pmc_dir, "c4__%s.json" % pmc_stamp.slug(kern))
            units = json.load(open(path)).get("units_per_dispatch") if b is not None else None
            per_ps[kern] = (b / units) if (b is not None and units) else None
            if kern == "estep_backward_kernel":
                rl.update(info)
        if per_ps.get("estep_backward_kernel") is not None:
            rl["traffic"] = int(round(per_ps["estep_backward_kernel"] * rl["sentences_per_launch"]))
            rl["traffic_per_sentence"] = per_ps["estep_backward_kernel"]
        if all(v is not None for v in per_ps.values()):
            names = {"unigram_fast_kernel<16, true, 4, true": "forward", "estep_backward_kernel": "backward",
                     "estep_compact_records_kernel": "compact_records", "estep_fold_kernel": "fold"}
            rl["pipeline_traffic_per_sentence"] = {names[k]: v for k, v in per_ps.items()}
    res.update({"value": psec, "sentences_per_s": total / psec, "ntok": pnt, "obj": pob,
                "epochs": args.estep_parity_epochs, "records_written": w1 - w0, "records_kept": k1 - k0,
                "records_note": "lattice-node records of the warm-up + timed epochs; kept = after dropping "
                                "provable no-ops (below a quarter ulp of a lower bound of their float "
                                "accumulator, estep_threshold_kernel)",
                "epoch_split": psplit, "repeat_epoch_bit_identical": prepeat, "roofline": rl})
    if world == 1 and not args.no_parity_check:
        res["check"] = parity_estep(args, buf, off, total, pieces, scores, T, pe, pob, pnt)
    if rank == 0 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        ns = args.estep_cpu_sample
        bb, oo = synth.normalized(ns, seed=7)
        b = bb.tobytes()
        sents = [b[int(oo[i]):int(oo[i + 1])] for i in range(ns)]
        th = min(args.cpu_threads, os.cpu_count() or 1)
        t0 = time.perf_counter()
        log("c4 cpu baseline")
        oracle_lib.estep(sents, np.ones(ns, dtype=np.int64), pieces, scores, th)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": total * dt / ns, "unit": "s/epoch (extrapolated)", "cores": th,
                               "kind": "port", "sample": "%d sentences, oracle RunEStep emulation with %d "
                               "threads, %.1f s wall, extrapolated to %d sentences" % (ns, th, dt, total)}
    dp.close()
    return res


if __name__ == "__main__":
    main()
