#!/bin/bash
# c2 kernel A/B: the bench's c2 leg (parity-checked at full size) with the
# tree's library and with each ablib/libspm_hip_<TAG>.so (SPM_AMD_LIB),
# alternating, two rounds.
# Usage (via gpurun): bash tools/gpu_r06_c2ab.sh OUT_TAG "TAG1 TAG2 ..." ["EXTRA_BENCH_ARGS"]
set -o pipefail
TAG=${1:-r06_c2ab}
OLDS=${2:-r06m}
EXTRA=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--steps 10 --warmup 3 --bpe-steps 0 --ja-lines 0 --estep-sentences 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats $EXTRA"
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py $A --detail $O/d.json > $O/tree_$i.json 2> $O/tree_$i.err || { echo "TREE FAILED"; tail -5 $O/tree_$i.err; exit 1; }
  for t in $OLDS; do
    SPM_AMD_LIB=$R/ablib/libspm_hip_$t.so timeout -k 10 300 python3 $R/bench.py $A --detail $O/d.json > $O/${t}_$i.json 2> $O/${t}_$i.err || { echo "$t FAILED"; tail -5 $O/${t}_$i.err; exit 1; }
  done
done
for f in $O/*_[12].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $f)', round(d['value']/1e9,4), 'G/s kernel_ms', round(r.get('kernel_ms'),4), 'parity', (d.get('parity') or {}))" 2>/dev/null || python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$(basename $f)', d['value'], d['legs'])"; done
