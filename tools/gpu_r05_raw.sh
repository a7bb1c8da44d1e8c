#!/bin/bash
# Fused raw-line path: coop + processor/CLI GPU tests, then the latency leg.
set -o pipefail
TAG=${1:-r05_raw}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_coop.py $R/tests/test_gpu_cli.py $R/tests/test_gpu_small_batch.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
L="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --estep-sentences 0 --ja-lines 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 300 python3 -u $R/bench.py $L > $O/lat.json 2> $O/lat.err || { echo "LAT FAILED"; tail -5 $O/lat.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/lat.json')); l=d.get('latency',{})
print({k: l.get(k) for k in ('encode_single_us','crossover_batch','c1_sentences_per_s')})
print([(b['batch'], b['us_per_call']) for b in l.get('batches', [])][:6])"
echo DONE
