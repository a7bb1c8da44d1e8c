#!/bin/bash
# All GPU tests, then the c5 leg.  Usage (via gpurun): bash tools/gpu_tests_c5.sh TAG
set -o pipefail
TAG=${1:-tests_c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest $R/tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash $R/tools/gpu_c5.sh $TAG
