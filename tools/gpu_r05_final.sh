#!/bin/bash
# Round-5 check: every GPU test, the default bench line (summary printed),
# then a rocprofv3 kernel trace of a short c2/c3 bench for profiles/.
# Usage (via gpurun): bash tools/gpu_r05_final.sh TAG
set -o pipefail
TAG=${1:-r05final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 900 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("c2 %.4g G/s kernel %.3f ms frac %.4f traffic %s" % (d["value"] / 1e9, r["kernel_ms"], r["frac"], r.get("traffic")))
b = d.get("bpe_c3", {})
print("c3 %.4g G/s kernel %.3f ms" % (b.get("value", 0) / 1e9, b.get("roofline", {}).get("kernel_ms", 0)))
j = d.get("ja_multibyte", {})
print("ja %.3g M/s" % (j.get("value", 0) / 1e6))
e = d.get("estep", {})
print("estep FAST", e.get("fast", {}).get("value"), "PARITY", e.get("value"), "roof", {k: e.get("roofline", {}).get(k) for k in ("kernel_ms", "frac", "traffic")})
t = d.get("train", {})
print("c5", t.get("value"), "peak", t.get("peak_device_bytes"), t.get("stage_peak_device_bytes"))
tb = d.get("train_bpe", {})
print("bpe train", tb.get("value"), {k: tb.get("stages", {}).get(k) for k in ("bpe_update_s", "total_s")})
l = d.get("latency", {})
print("latency single", l.get("encode_single_us"), "crossover", l.get("crossover_batch"), [(x["batch"], x["us_per_call"]) for x in l.get("batches", [])][:4])
print("c1 botchan", l.get("c1_botchan", {}).get("encode_single_us"), "us/line", l.get("c1_botchan", {}).get("line_by_line_sentences_per_s"), "lines/s")
print("e2e_raw", d.get("e2e_raw", {}).get("value"))
print("parity", {k: (v.get("mismatches") if isinstance(v, dict) else v) for k, v in d.get("parity", {}).items()})
print("peak bytes/rank", d.get("peak_device_bytes_per_rank"))
PY
P3="--steps 2 --warmup 1 --sentences 10000000 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --ja-lines 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $P3 > $O/trace.json 2> $O/trace.log || { echo "TRACE FAILED"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace_c2c3.txt > /dev/null
head -8 $O/kernel_trace_c2c3.txt
find $O -name '*.db' -delete
echo DONE
