#!/bin/bash
# Device corpus load: 100M-line spm_train (device and host load), then the
# trainer GPU tests with the device load on.  Usage: bash tools/gpu_devload_check.sh TAG
set -o pipefail
TAG=${1:-devload}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
bash $R/tools/gpu_c5_debug.sh $TAG 100000000 || exit 1
SPM_HIP_DEVICE_LOAD=1 timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_train.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/train_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/train_tests.log; exit 1; }
tail -2 $O/train_tests.log
