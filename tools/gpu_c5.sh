#!/bin/bash
# c5 leg only (spm_train unigram 32k on 100M synthetic lines), stage breakdown.
# Usage (via gpurun): bash tools/gpu_c5.sh TAG [bench args...]
set -o pipefail
TAG=${1:-c5}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C5="--steps 1 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --estep-sentences 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 600 python3 -u $R/bench.py $C5 "$@" > $O/c5.json 2> $O/c5.err || { echo "C5 FAILED"; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); t=d.get('train'); print(json.dumps(t['stages']))"
echo DONE
