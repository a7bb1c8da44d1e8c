#!/bin/bash
# E-step chunk-size A/B (SPM_HIP_ESTEP_CHUNK = max sentences per chunk; the
# call is cut into equal chunks of at most that size).  c4 legs only.
# Usage (via gpurun): bash tools/gpu_chunk_ab.sh TAG
set -o pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 3"
for C in 4194304 6400000 13000000 2600000 4194304; do
  SPM_HIP_ESTEP_CHUNK=$C timeout -k 10 240 python3 -u $R/bench.py $ARGS > $O/chunk_$C.json 2> $O/chunk_$C.err || { echo "CHUNK $C FAILED"; tail -5 $O/chunk_$C.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['estep']; print(sys.argv[2], 'FAST', round(d['value'],4), 'PARITY', round(d['parity']['value'],4))" $O/chunk_$C.json $C | tee -a $O/chunk_ab.txt
done
echo DONE
