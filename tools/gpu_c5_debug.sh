#!/bin/bash
# spm_train on N synthetic lines with the trainer's log streamed to a file
# (device load, then the host load).  Usage: bash tools/gpu_c5_debug.sh TAG LINES
set -o pipefail
TAG=${1:-c5dbg}; N=${2:-10000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
SPM_HIP_DEVICE_LOAD=1 timeout -k 10 240 python3 -u $R/tools/train_bench.py --lines $N --workers 8 --log $O/train_dev.log > $O/dev.json 2> $O/dev.err; echo "dev rc=$?"; tail -3 $O/train_dev.log; cat $O/dev.json
timeout -k 10 240 python3 -u $R/tools/train_bench.py --lines $N --workers 8 --log $O/train_host.log > $O/host.json 2> $O/host.err; echo "host rc=$?"; cat $O/host.json
grep -h "LoadSentences\|ReadTextDevice\|Loaded" $O/train_dev.log $O/train_host.log
