#!/bin/bash
# Trainer GPU tests, then the c5 leg.  Usage (via gpurun): bash tools/gpu_train_tests_c5.sh TAG
set -o pipefail
TAG=${1:-train_c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_train.py $R/tests/test_gpu_scratch_cache.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash $R/tools/gpu_c5.sh $TAG
cd /tmp && export TMPDIR=/tmp
C5="--steps 1 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --estep-sentences 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $C5 > $O/trace.json 2> $O/trace.log || { echo "TRACE FAILED"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $O/trace/run_results.db $O/kernel_trace_c5.txt > /dev/null
head -30 $O/kernel_trace_c5.txt
find $O -name '*.db' -delete
