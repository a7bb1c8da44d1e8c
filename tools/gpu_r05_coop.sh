#!/bin/bash
# Cooperative-kernel check: coop + parity GPU tests, then the Japanese leg
# (1 M lines of wagahaiwa, full-size parity) with coop on / off.
set -o pipefail
TAG=${1:-r05_coop}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_coop.py $R/tests/test_gpu_parity.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
JA="--steps 3 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats"
for v in 1 0; do
  SPM_HIP_COOP=$v timeout -k 10 400 python3 -u $R/bench.py $JA > $O/ja_coop$v.json 2> $O/ja_coop$v.err || { echo "JA FAILED"; tail -5 $O/ja_coop$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ja_coop$v.json')); j=d.get('ja_multibyte',{}); print('coop=$v ja', j.get('value'), j.get('ms_per_step'), d.get('parity',{}).get('ja_multibyte'))"
done
