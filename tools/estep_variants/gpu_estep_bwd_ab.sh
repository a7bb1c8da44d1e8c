#!/bin/bash
# E-step kernel variants (env var $3, default SPM_HIP_ESTEP_BWD): parity tests, then
# bench's c4 leg (FAST + PARITY s/epoch) per variant.
set -o pipefail
TAG=${1:-estep_bwd}; V=${2:-"0 1 3 7"}; VAR=${3:-SPM_HIP_ESTEP_BWD}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for B in $V; do
  env $VAR=$B timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_estep.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_$B.log 2>&1 || { echo "TESTS $B FAILED"; tail -30 $O/tests_$B.log; exit 1; }
  echo "$VAR=$B: $(tail -1 $O/tests_$B.log)"
done
ARGS="--steps 1 --warmup 1 --bpe-steps 0 --raw-steps 0 --train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 2"
for B in $V; do
  env $VAR=$B timeout -k 10 300 python3 $R/bench.py $ARGS > $O/bench_$B.json 2> $O/bench_$B.err || { echo "BENCH $B FAILED"; tail -5 $O/bench_$B.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/bench_$B.json')); e=d['estep']; print('$VAR=$B: FAST %.4f s/epoch, PARITY %.4f s/epoch, obj %s / %s' % (e['value'], e['parity']['value'], e['obj'], e['parity']['obj']))"
done
echo DONE
