# Kernel trace of the c4 E-step legs only (FAST + PARITY, one epoch each).
set -o pipefail
TAG=${1:-estep}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --sentences 1000000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check --estep-epochs 1 --estep-parity-epochs 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $ARGS > $O/bench.json 2> $O/trace.log || { echo TRACE FAILED; tail -5 $O/trace.log; exit 1; }
tail -c 600 $O/bench.json
echo DONE
