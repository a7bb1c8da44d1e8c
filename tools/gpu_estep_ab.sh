#!/bin/bash
# E-step A/B round trip: E-step + trainer GPU tests (bit-exact vs the
# oracle), then the c4 leg (FAST + PARITY, 100M sentences/epoch) under each
# value of an env knob.  Usage (via gpurun): bash tools/gpu_estep_ab.sh TAG KNOB v1 v2 ...
set -o pipefail
TAG=${1:-estep}; KNOB=${2:-SPM_HIP_ESTEP_WPE}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_estep.py $R/tests/test_gpu_dist_estep.py $R/tests/test_gpu_train.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ES="--bpe-steps 0 --raw-steps 0 --steps 1 --warmup 1 --sentences 1000000 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 2 --ja-lines 0 --latency-calls 0 --no-parity-check"
for v in "$@"; do
  env $KNOB=$v timeout -k 10 400 python3 -u $R/bench.py $ES > $O/estep_$v.json 2> $O/estep_$v.err || { echo "ESTEP FAILED"; tail -5 $O/estep_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/estep_$v.json'))['estep']; print('$KNOB=$v FAST', d['value'], 'PARITY', d['parity']['value'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $ES > $O/trace.json 2> $O/trace.log || { echo "TRACE FAILED"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace.txt > /dev/null
head -14 $O/kernel_trace.txt
find $O -name '*.db' -delete
echo DONE
