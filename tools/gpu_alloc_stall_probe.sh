#!/bin/bash
# Does seed mining's hipMalloc stall after another process freed a large
# amount of device memory?  c5 spm_train once on a fresh process, then right
# after a process that fills and frees GB_FILL GB, then after a 20 s pause.
# Usage: bash tools/gpu_alloc_stall_probe.sh TAG [GB_FILL] ["GB_FILL2 ..."] [SLEEP_S]
# (GB_FILL2 / SLEEP_S: an extra after-fill run with another fill size, and one
# with a pause of SLEEP_S seconds between the fill and the train.)
set -o pipefail
TAG=${1:-stall}; GB=${2:-200}; GB2=${3:-0}; SL=${4:-0}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
D=$(mktemp -d /tmp/stall_XXXX)
timeout -k 10 200 python3 -u -c "
import sys; sys.path.insert(0, '$R/tools')
import train_bench
train_bench.write_corpus('$D/corpus.txt', 100000000, 1234, workers=8)
" 2> $O/gen.log || { echo "GEN FAILED"; exit 1; }
run() {
  echo "== $1" >> $O/runs.log
  timeout -k 10 120 $R/sentencepiece-comments_amd/lib/spm_train --input=$D/corpus.txt --model_prefix=$D/m --model_type=unigram --vocab_size=32000 --normalization_rule_name=identity --num_threads=16 --timings > $O/t_$1.json 2> $O/l_$1.log || { echo "TRAIN $1 FAILED"; exit 1; }
  echo "$1 $(grep -o '"seed_s": [0-9.]*' $O/t_$1.json) $(grep -o '"seed_stages_ms": [^]]*' $O/t_$1.json) $(grep -o '"total_s": [0-9.]*' $O/t_$1.json)"
}
fill() {
  local gb=${1:-$GB}
  timeout -k 10 120 python3 -c "
import torch, time
t0 = time.time()
xs = [torch.ones(1 << 30, dtype=torch.uint8, device='cuda') for _ in range($gb)]
torch.cuda.synchronize()
print('filled', len(xs), 'GB in', round(time.time() - t0, 2), 's')
" || { echo "FILL FAILED"; exit 1; }
}
run fresh
fill
run after_fill
fill
sleep 20
run after_fill_20s
for g in $GB2; do [ "$g" != 0 ] && { fill $g; run after_fill_$g; sleep 20; }; done
if [ "$SL" != 0 ]; then fill; sleep $SL; run after_fill_${SL}s; sleep 20; fi
run again
rm -rf $D
