#!/bin/bash
# c4 PARITY E-step A/B: the bench's E-step leg (one 100 M-sentence epoch after
# a warm-up epoch) with the tree's library and with each
# ablib/libspm_hip_<TAG>.so (SPM_AMD_LIB), alternating, two rounds.
# Usage (via gpurun): bash tools/gpu_r06_c4ab.sh OUT_TAG "TAG1 ..."
set -o pipefail
TAG=${1:-r06_c4ab}
OLDS=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --ja-lines 0 --estep-sentences 100000000 --estep-parity-epochs 2 --estep-warmup 1 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py $A --detail $O/d.json > $O/tree_$i.json 2> $O/tree_$i.err || { echo "TREE FAILED"; tail -5 $O/tree_$i.err; exit 1; }
  for t in $OLDS; do
    SPM_AMD_LIB=$R/ablib/libspm_hip_$t.so timeout -k 10 300 python3 $R/bench.py $A --detail $O/d.json > $O/${t}_$i.json 2> $O/${t}_$i.err || { echo "$t FAILED"; tail -5 $O/${t}_$i.err; exit 1; }
  done
done
for f in $O/*_[12].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$(basename $f)', d['legs'].get('c4'))"; done
