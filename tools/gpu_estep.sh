# E-step round trip: E-step/trainer tests, FAST+PARITY bench leg, kernel trace.
set -o pipefail
TAG=${1:-estep}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_estep.py $R/tests/test_gpu_train.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ARGS="--steps 2 --warmup 1 --sentences 1000000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 1 --estep-parity-epochs 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $ARGS > $O/bench.json 2> $O/trace.log || { echo TRACE FAILED; tail -5 $O/trace.log; exit 1; }
tail -c 700 $O/bench.json
echo DONE
