#!/bin/bash
# Japanese-leg A/B (bench.py's ja leg, full-size parity on): the tree's
# library vs ablib/libspm_hip_<OLD>.so (SPM_AMD_LIB), alternating, after
# optional GPU tests.
# Usage (via gpurun): bash tools/gpu_r06_jaab.sh TAG OLD ["TESTS"]
set -o pipefail
TAG=${1:-r06_jaab}
OLD=${2:-r06jj}
TESTS=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  (cd $R && timeout -k 10 800 python3 -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread) > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -30; tail -20 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
A="--steps 5 --warmup 2 --sentences 100000 --bpe-steps 0 --estep-sentences 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats"
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py $A --detail $O/d.json > $O/tree_$i.json 2> $O/tree_$i.err || { echo "TREE FAILED"; tail -5 $O/tree_$i.err; exit 1; }
  SPM_AMD_LIB=$R/ablib/libspm_hip_$OLD.so timeout -k 10 300 python3 $R/bench.py $A --detail $O/d.json > $O/old_$i.json 2> $O/old_$i.err || { echo "OLD FAILED"; tail -5 $O/old_$i.err; exit 1; }
done
for f in tree_1 old_1 tree_2 old_2; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['legs'].get('ja'), d.get('parity') or '')"; done
