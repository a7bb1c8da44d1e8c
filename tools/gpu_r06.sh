#!/bin/bash
# Round-6 GPU step: selected GPU tests, then an optional bench run (its JSON
# line kept, a summary printed).  Every GPU step has its own time limit and
# the script stops at the first failure.
# Usage (via gpurun): bash tools/gpu_r06.sh TAG "TEST_ARGS" "BENCH_ARGS"
#   TEST_ARGS  pytest selection ("" = skip tests, "all" = every GPU test)
#   BENCH_ARGS bench.py arguments ("" = skip the bench, "default" = none)
set -o pipefail
TAG=${1:-r06}
TESTS=${2:-}
BENCH=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  SEL="$TESTS"
  [ "$TESTS" = "all" ] && SEL="$R/tests"
  (cd $R && timeout -k 10 1000 python3 -u -m pytest $SEL -x -v -m gpu --timeout 300 --timeout-method thread) > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" $O/gpu_tests.log | head -30; tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
if [ -n "$BENCH" ]; then
  [ "$BENCH" = "default" ] && BENCH=""
  timeout -k 10 1000 python3 -u $R/bench.py $BENCH > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
  python3 $R/tools/bench_summary.py $O/bench.json
fi
echo DONE
