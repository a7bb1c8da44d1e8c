set -o pipefail
mkdir -p gpurun_out/r02f
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_train.py -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/r02f/tests.log 2>&1 || { tail -40 $R/gpurun_out/r02f/tests.log; exit 1; }
tail -3 $R/gpurun_out/r02f/tests.log
timeout -k 10 400 python3 $R/bench.py --steps 5 --warmup 2 --bpe-steps 0 --raw-steps 0 --train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 1 --estep-parity-epochs 1 > $R/gpurun_out/r02f/bench.json 2> $R/gpurun_out/r02f/bench.err || { tail -20 $R/gpurun_out/r02f/bench.err; exit 1; }
cat $R/gpurun_out/r02f/bench.json
