# c5 at 100M lines (unigram) and a 10M-line BPE train, timings JSON to gpurun_out.
set -o pipefail
TAG=${1:-train}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u $R/tools/train_bench.py --lines 100000000 > $O/train_c5_100m.json 2> $O/train_c5_100m.log || { tail -5 $O/train_c5_100m.log; exit 1; }
cat $O/train_c5_100m.json
timeout -k 10 400 python3 -u $R/tools/train_bench.py --lines 10000000 --args "--model_type=bpe --normalization_rule_name=identity --num_threads=16" > $O/train_bpe_10m.json 2> $O/train_bpe_10m.log || { tail -5 $O/train_bpe_10m.log; exit 1; }
cat $O/train_bpe_10m.json
echo DONE
