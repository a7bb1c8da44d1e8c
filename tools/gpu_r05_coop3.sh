#!/bin/bash
# Cooperative kernel (one-round Viterbi reads, select-only candidate fold,
# backtrace block prefetch): coop / parity / small-batch GPU tests, the
# Japanese leg with full parity (then with phase cycles), and the per-call
# latency probe.
set -o pipefail
TAG=${1:-r05_coop3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_coop.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_small_batch.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
JA="--steps 3 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats"
timeout -k 10 400 python3 -u $R/bench.py $JA > $O/ja.json 2> $O/ja.err || { echo "JA FAILED"; tail -5 $O/ja.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ja.json')); j=d.get('ja_multibyte',{}); print('ja', round(j.get('value')/1e6,2), 'M/s', round(j.get('ms_per_step'),2), 'ms', d.get('parity',{}).get('ja_multibyte',{}).get('mismatches'))"
SPM_HIP_COOP_PROF=1 timeout -k 10 400 python3 -u $R/bench.py $JA > $O/ja_prof.json 2> $O/ja_prof.err || { echo "JA PROF FAILED"; tail -5 $O/ja_prof.err; exit 1; }
grep "coop prof" $O/ja_prof.err | tail -1
timeout -k 10 300 python3 -u $R/tools/raw_latency_probe.py > $O/lat.txt 2>&1 || { echo PROBE FAILED; tail -5 $O/lat.txt; exit 1; }
grep -v amdgpu.ids $O/lat.txt
echo DONE
