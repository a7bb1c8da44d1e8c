#!/bin/bash
# E-step A/B over env settings: the E-step GPU tests under TEST_ENV (bit-exact
# vs the oracle), then the c4 leg (FAST + PARITY, 100M sentences/epoch) under
# each setting.  Usage (via gpurun):
#   bash tools/gpu_env_ab.sh TAG "TEST_ENV" "ENV1" "ENV2" ...   (ENV = "K=v K2=v2", or "-" for none)
set -o pipefail
TAG=${1:-envab}; TEST_ENV=${2:--}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ev() { [ "$1" = "-" ] && echo "" || echo "$1"; }
env $(ev "$TEST_ENV") timeout -k 10 600 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_estep.py $R/tests/test_gpu_dist_estep.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ES="--bpe-steps 0 --raw-steps 0 --steps 1 --warmup 1 --sentences 1000000 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 2 --ja-lines 0 --latency-calls 0 --no-parity-check"
i=0
for v in "$@"; do
  i=$((i+1))
  env $(ev "$v") timeout -k 10 400 python3 -u $R/bench.py $ES > $O/estep_$i.json 2> $O/estep_$i.err || { echo "ESTEP FAILED"; tail -5 $O/estep_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/estep_$i.json'))['estep']; print('$v', 'FAST', d['value'], 'PARITY', d['parity']['value'])"
done
echo DONE
