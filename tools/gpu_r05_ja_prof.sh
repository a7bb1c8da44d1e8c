#!/bin/bash
# Kernel trace of the Japanese leg (cooperative kernel on).
set -o pipefail
TAG=${1:-r05_ja_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
JA="--steps 3 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $JA > $O/ja.json 2> $O/trace.log || { tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace.txt > /dev/null
head -24 $O/kernel_trace.txt
find $O -name '*.db' -delete
