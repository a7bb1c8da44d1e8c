set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r02u
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_train.py -x -v -m gpu -k bpe --timeout 300 --timeout-method thread > $R/gpurun_out/r02u/tests.log 2>&1 || { tail -30 $R/gpurun_out/r02u/tests.log; exit 1; }
tail -1 $R/gpurun_out/r02u/tests.log
timeout -k 10 400 python3 -u $R/tools/train_bench.py --lines 10000000 --args "--model_type=bpe --normalization_rule_name=identity --num_threads=16" > $R/gpurun_out/r02u/train_bpe_10m.json 2> $R/gpurun_out/r02u/train_bpe_10m.log || { tail -5 $R/gpurun_out/r02u/train_bpe_10m.log; exit 1; }
cat $R/gpurun_out/r02u/train_bpe_10m.json
