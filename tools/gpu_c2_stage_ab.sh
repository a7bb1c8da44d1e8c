#!/bin/bash
# c2 kernel variant A/B: unigram parity tests on the variant build, then
# alternating c2 bench legs (in-tree library vs lib/<var>), then the
# WRITE/FETCH passes of both.  Usage: bash tools/gpu_c2_stage_ab.sh TAG VAR
set -o pipefail
TAG=${1:-c2stage}; VAR=${2:-stage}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
VL=$R/sentencepiece-comments_amd/lib/$VAR/libspm_hip.so
SPM_AMD_LIB=$VL timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_async.py $R/tests/test_gpu_small_batch.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
C2="--steps 20 --warmup 3 --bpe-steps 0 --raw-steps 0 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats"
for k in 1 2; do
  for v in base $VAR; do
    if [ $v = base ]; then L=""; else L=$VL; fi
    SPM_AMD_LIB=$L timeout -k 10 300 python3 -u $R/bench.py $C2 > $O/c2_${v}_$k.json 2> $O/c2_${v}_$k.err || { echo "C2 $v FAILED"; tail -5 $O/c2_${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c2_${v}_$k.json')); print('$v', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'parity', d.get('parity_check', {}).get('mismatches'))"
  done
done
bash $R/tools/gpu_c2_write_ab.sh ${TAG}_w $VAR
