#!/bin/bash
# Kernel trace of spm_train on N synthetic lines (c5): the corpus is written
# first, then rocprofv3 runs lib/spm_train itself.  Usage: bash tools/gpu_c5_trace.sh TAG N
set -o pipefail
TAG=${1:-c5trace}; N=${2:-100000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
D=$(mktemp -d /tmp/c5t_XXXX)
timeout -k 10 200 python3 -u -c "
import sys; sys.path.insert(0, '$R/tools')
import train_bench
train_bench.write_corpus('$D/corpus.txt', $N, 1234, workers=8)
" 2> $O/gen.log || { echo "GEN FAILED"; tail -3 $O/gen.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $R/sentencepiece-comments_amd/lib/spm_train --input=$D/corpus.txt --model_prefix=$D/m --model_type=unigram --vocab_size=32000 --normalization_rule_name=identity --num_threads=16 --timings > $O/timings.json 2> $O/train.log || { echo "TRACE FAILED"; tail -5 $O/train.log; exit 1; }
cat $O/timings.json
python3 $R/tools/rocprof_summary.py $O/trace/run_results.db $O/kernel_trace_c5.txt > /dev/null
head -40 $O/kernel_trace_c5.txt
find $O -name '*.db' -delete
# Load A/B: READERS_AB="readers:piece_mb ..." (the corpus is in the page cache either way).
for ab in ${READERS_AB:-}; do
  rd=${ab%%:*}; mb=${ab##*:}
  SPM_HIP_LOAD_READERS=$rd SPM_HIP_LOAD_PIECE_MB=$mb timeout -k 10 120 $R/sentencepiece-comments_amd/lib/spm_train --input=$D/corpus.txt --model_prefix=$D/m --model_type=unigram --vocab_size=32000 --normalization_rule_name=identity --num_threads=16 --timings > $O/timings_load_${rd}_$mb.json 2> $O/train_load_${rd}_$mb.log || { echo "LOAD $ab FAILED"; exit 1; }
  echo "readers=$rd piece_mb=$mb $(grep -o 'file to HBM [0-9.]* s' $O/train_load_${rd}_$mb.log) $(grep -o '"total_s": [0-9.]*' $O/timings_load_${rd}_$mb.json)"
done
# Env A/B: ENV_AB="VAR=VAL ..." one timing run each.
for ev in ${ENV_AB:-}; do
  env $ev timeout -k 10 120 $R/sentencepiece-comments_amd/lib/spm_train --input=$D/corpus.txt --model_prefix=$D/m --model_type=unigram --vocab_size=32000 --normalization_rule_name=identity --num_threads=16 --timings > $O/timings_env.json 2> $O/train_env.log || { echo "ENV $ev FAILED"; exit 1; }
  echo "$ev $(grep -o '"seed_s": [0-9.]*' $O/timings_env.json) $(grep -o '"seed_stages_ms": [^]]*' $O/timings_env.json) $(grep -o '"total_s": [0-9.]*' $O/timings_env.json)"
done
rm -rf $D
