#!/bin/bash
# BPE lane kernel with staged output: the full GPU suite, the c3 leg, and PMC
# traffic (FETCH / WRITE) of bpe_lane_kernel + bpe_compact_kernel; then the
# E-step PMC passes (PARITY backward kernel per-dispatch traffic) that bench.py
# reads from profiles/.
set -o pipefail
TAG=${1:-r05_bpe}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $R/tests > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--steps 5 --warmup 2 --sentences 10000000 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --ja-lines 0 --no-cpu-baseline --no-probe-stats"
timeout -k 10 400 python3 -u $R/bench.py $C3 > $O/c3.json 2> $O/c3.err || { echo "C3 FAILED"; tail -5 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); b=d['bpe_c3']; print('c2', d['value'], 'c3', b['value'], b['roofline']['kernel_ms'], d.get('parity',{}).get('c3'))"
P3="--steps 2 --warmup 1 --sentences 10000000 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --ja-lines 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $P3 > $O/trace.json 2> $O/trace.log || { echo "TRACE FAILED"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace.txt > /dev/null
head -12 $O/kernel_trace.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 $R/bench.py $P3 > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 $R/bench.py $P3 > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -5 $O/pmc_write.log; exit 1; }
for k in "bpe_lane_kernel" "bpe_compact_kernel" "unigram_fast_kernel<16, true, 7"; do
  python3 $R/tools/pmc_traffic.py $(find $O/pmc_fetch -name '*results.db' | head -1) $(find $O/pmc_write -name '*results.db' | head -1) "$k" $O/pmc_$(echo $k | tr -cd 'a-z0-9_').json | grep -E "kernel_substr|hbm_read_bytes_per_launch|hbm_write_bytes_per_launch"
done
find $O -name '*.db' -delete
EST="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check --estep-sentences 12500000 --estep-epochs 1 --estep-warmup 0 --estep-parity-epochs 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/epmc_fetch -o run -- python3 $R/bench.py $EST > $O/epmc_fetch.log 2>&1 || { echo "E PMC FETCH FAILED"; tail -5 $O/epmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/epmc_write -o run -- python3 $R/bench.py $EST > $O/epmc_write.log 2>&1 || { echo "E PMC WRITE FAILED"; tail -5 $O/epmc_write.log; exit 1; }
for k in "estep_backward_kernel<16, 3, 8>" "estep_backward_kernel<16, 4," "estep_forward" "estep_compact_records" "estep_fold_kernel"; do
  python3 $R/tools/pmc_traffic.py $(find $O/epmc_fetch -name '*results.db' | head -1) $(find $O/epmc_write -name '*results.db' | head -1) "$k" $O/epmc_$(echo $k | tr -cd 'a-z0-9_').json | grep -E "kernel_substr|dispatches|hbm_read_bytes_per_launch|hbm_write_bytes_per_launch"
done
find $O -name '*.db' -delete
echo DONE
