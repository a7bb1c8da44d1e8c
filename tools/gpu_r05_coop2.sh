#!/bin/bash
# Cooperative kernel (register backtrace) + BPE lane setup: coop, parity,
# small-batch GPU tests; the Japanese leg with full parity and phase cycles;
# c3 with full parity.
set -o pipefail
TAG=${1:-r05_coop2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_coop.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_small_batch.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
JA="--steps 3 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats"
SPM_HIP_COOP_PROF=1 timeout -k 10 400 python3 -u $R/bench.py $JA > $O/ja.json 2> $O/ja.err || { echo "JA FAILED"; tail -5 $O/ja.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ja.json')); j=d.get('ja_multibyte',{}); print('ja', round(j.get('value')/1e6,2), 'M/s', round(j.get('ms_per_step'),2), 'ms', d.get('parity',{}).get('ja_multibyte',{}).get('mismatches'))"
grep "coop prof" $O/ja.err | tail -2
C3="--steps 5 --warmup 2 --sentences 10000000 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --ja-lines 0 --no-cpu-baseline --no-probe-stats"
timeout -k 10 400 python3 -u $R/bench.py $C3 > $O/c3.json 2> $O/c3.err || { echo "C3 FAILED"; tail -5 $O/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3.json')); b=d['bpe_c3']; print('c2', round(d['value']/1e6,1), 'c3', round(b['value']/1e6,1), b['roofline']['kernel_ms'], d.get('parity',{}).get('c3',{}).get('mismatches'), d.get('parity',{}).get('c2',{}).get('mismatches'))"
echo DONE
