# Encode round trip: parity tests + c2 bench leg + kernel trace of it.
set -o pipefail
TAG=${1:-enc}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_spt.py $R/tests/test_gpu_concurrency.py $R/tests/test_gpu_cli.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ARGS="--bpe-steps 0 --raw-steps 0 --train-lines 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats"
timeout -k 10 300 python3 $R/bench.py $ARGS > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py --steps 3 --warmup 1 $ARGS > $O/trace.log 2>&1 || { echo TRACE FAILED; exit 1; }
echo DONE
