#!/bin/bash
# c3 (BPE encode) A/B of an env knob, alternating values; BPE GPU tests first.
# Usage (via gpurun): bash tools/gpu_ab_c3.sh TAG KNOB v1 v2 ...
set -o pipefail
TAG=${1:-ab_c3}; KNOB=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
[ -n "$NOTEST" ] || timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_parity.py $R/tests/test_gpu_small_batch.py -k "bpe or BPE" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C3="--steps 5 --warmup 2 --sentences 10000000 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --ja-lines 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
k=0
for v in "$@"; do
  k=$((k+1))
  env $KNOB=$v timeout -k 10 300 python3 -u $R/bench.py $C3 > $O/c3_${k}_$v.json 2> $O/c3_${k}_$v.err || { echo "C3 FAILED"; tail -5 $O/c3_${k}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_${k}_$v.json')); b=d['bpe_c3']; print('$KNOB=$v c3', round(b['value']/1e6,1), 'M/s kernel_ms', round(b['roofline']['kernel_ms'],3))"
done
echo DONE
