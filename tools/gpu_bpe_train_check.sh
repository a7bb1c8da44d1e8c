#!/bin/bash
# Trainer GPU tests, then spm_train --model_type=bpe on N synthetic lines
# (bench.py's train_bpe leg, default 10 M) with --timings, twice.
# Usage: bash tools/gpu_bpe_train_check.sh TAG [N]
set -o pipefail
TAG=${1:-bpetrain}; N=${2:-10000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_train.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
D=$(mktemp -d /tmp/bpe_XXXX)
timeout -k 10 200 python3 -u -c "
import sys; sys.path.insert(0, '$R/tools')
import train_bench
train_bench.write_corpus('$D/corpus.txt', $N, 1234, workers=8)
" 2> $O/gen.log || { echo "GEN FAILED"; tail -3 $O/gen.log; exit 1; }
k=0
for ev in ${ENV_AB:-NONE=0 NONE=0}; do
  k=$((k+1))
  env $ev timeout -k 10 120 $R/sentencepiece-comments_amd/lib/spm_train --input=$D/corpus.txt --model_prefix=$D/m --model_type=bpe --vocab_size=32000 --normalization_rule_name=identity --num_threads=16 --timings > $O/timings_$k.json 2> $O/train_$k.log || { echo "TRAIN FAILED"; tail -5 $O/train_$k.log; exit 1; }
  echo "run $k $ev $(grep -o '"total_s": [0-9.]*' $O/timings_$k.json) $(grep -o '"bpe_update_s": [0-9.]*' $O/timings_$k.json) $(grep -o '"bpe_update_sort_s": [0-9.]*' $O/timings_$k.json) $(grep -o '"bpe_update_replays": [0-9]*' $O/timings_$k.json)"
done
rm -rf $D
