#!/bin/bash
# New GPU tests of this step (scratch cache selftest, split fallback) then the
# E-step counter passes.  Usage (via gpurun): bash tools/gpu_r04_misc.sh TAG
set -o pipefail
TAG=${1:-r04_misc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_scratch_cache.py $R/tests/test_gpu_train.py -x -v -m gpu --timeout 300 --timeout-method thread -k "scratch or split or node_capacity or seed" > $R/gpurun_out/$TAG/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $R/gpurun_out/$TAG/tests.log; exit 1; }
tail -3 $R/gpurun_out/$TAG/tests.log
bash $R/tools/gpu_r04_estep_pmc.sh $TAG
