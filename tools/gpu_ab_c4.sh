#!/bin/bash
# c4 (E-step) A/B of an env knob, alternating values (no tests: timing only).
set -o pipefail
TAG=${1:-ab_c4}; KNOB=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ES="--bpe-steps 0 --raw-steps 0 --steps 1 --warmup 1 --sentences 100000 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 1 --estep-parity-epochs 2 --ja-lines 0 --latency-calls 0 --no-parity-check"
k=0
for v in "$@"; do
  k=$((k+1))
  env $KNOB=$v timeout -k 10 300 python3 -u $R/bench.py $ES > $O/e_${k}_$v.json 2> $O/e_${k}_$v.err || { echo "C4 FAILED"; tail -5 $O/e_${k}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/e_${k}_$v.json'))['estep']; r=d['parity']['roofline']; print('$KNOB=$v PARITY', round(d['parity']['value'],4), 'fwd', round(r['forward_kernel_ms'],3), 'bwd', round(r['kernel_ms'],3))"
done
echo DONE
