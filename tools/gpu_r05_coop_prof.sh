#!/bin/bash
# Cooperative kernel phase cycles (SPM_HIP_COOP_PROF) on the Japanese leg.
set -o pipefail
TAG=${1:-r05_coop_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
JA="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
SPM_HIP_COOP_PROF=1 timeout -k 10 300 python3 -u $R/bench.py $JA > $O/ja.json 2> $O/ja.err || { tail -5 $O/ja.err; exit 1; }
grep "coop prof" $O/ja.err | tail -3
