#!/bin/bash
# E-step + trainer GPU tests, then the c5 kernel trace.  Usage: bash tools/gpu_estep_train_check.sh TAG
set -o pipefail
TAG=${1:-estrain}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_estep.py $R/tests/test_gpu_train.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash $R/tools/gpu_c5_trace.sh $TAG 100000000
