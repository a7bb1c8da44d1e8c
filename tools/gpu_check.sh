#!/bin/bash
# One GPU round trip: parity tests, bench, kernel trace and HBM PMC passes.
# Usage (via gpurun): bash tools/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 $R/bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
# Kernel trace of every leg but c5 (its own process) with short step counts.
SHORT="--steps 3 --warmup 1 --bpe-steps 2 --raw-steps 2 --estep-epochs 1 --estep-parity-epochs 1 --train-lines 0 --no-cpu-baseline --no-probe-stats"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $SHORT "$@" > $O/trace.log 2>&1 || { echo "TRACE FAILED"; exit 1; }
# HBM traffic of the encode kernels (c2 + c3 legs only).
ENC="--steps 2 --warmup 1 --bpe-steps 2 --raw-steps 0 --estep-sentences 0 --train-lines 0 --no-cpu-baseline --no-probe-stats"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 $R/bench.py $ENC "$@" > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 $R/bench.py $ENC "$@" > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; exit 1; }
echo DONE
