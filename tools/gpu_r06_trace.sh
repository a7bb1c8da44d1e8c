#!/bin/bash
# rocprofv3 kernel trace (--kernel-trace --stats) of chosen bench legs, each
# summarised into a text table (tools/rocprof_summary.py) for profiles/.
# Usage (via gpurun): bash tools/gpu_r06_trace.sh TAG "LEGS"   (LEGS: enc ja c4)
set -o pipefail
TAG=${1:-r06_trace}
LEGS=${2:-"enc ja c4"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
OFF="--raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
for leg in $LEGS; do
  case $leg in
    enc) A="--steps 3 --warmup 1 --sentences 10000000 --bpe-steps 3 --ja-lines 0 --estep-sentences 0 $OFF" ;;
    ja)  A="--steps 3 --warmup 1 --sentences 100000 --bpe-steps 0 --estep-sentences 0 $OFF" ;;
    c4)  A="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --ja-lines 0 --estep-sentences 100000000 --estep-parity-epochs 1 --estep-warmup 1 $OFF" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$leg -o run -- python3 $R/bench.py $A --detail $O/$leg.detail.json > $O/$leg.json 2> $O/$leg.log || { echo "TRACE $leg FAILED"; tail -5 $O/$leg.log; exit 1; }
  python3 $R/tools/rocprof_summary.py $(find $O/$leg -name '*results.db' | head -1) $O/kernel_trace_$leg.txt > /dev/null
  head -16 $O/kernel_trace_$leg.txt
done
find $O -name '*.db' -delete
echo DONE
