#!/bin/bash
# Trainer round trip: the trainer GPU tests (unigram + BPE, bit-exact vs the
# oracle), the 10M-line BPE train with its merge-loop stage times and the
# c5 100M-line unigram train with its stages.
# Usage (via gpurun): bash tools/gpu_train_check.sh TAG
set -o pipefail
TAG=${1:-train}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_train.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 -u $R/tools/train_bench.py --lines 10000000 --model-type bpe --workers 16 --args "--normalization_rule_name=identity --num_threads=16" > $O/train_bpe_10m.json 2> $O/train_bpe_10m.log || { echo "BPE TRAIN FAILED"; tail -5 $O/train_bpe_10m.log; exit 1; }
cat $O/train_bpe_10m.json
timeout -k 10 600 python3 -u $R/tools/train_bench.py --lines 100000000 --model-type unigram --workers 16 --args "--normalization_rule_name=identity --num_threads=16" > $O/train_c5_100m.json 2> $O/train_c5_100m.log || { echo "C5 TRAIN FAILED"; tail -5 $O/train_c5_100m.log; exit 1; }
cat $O/train_c5_100m.json
echo DONE
