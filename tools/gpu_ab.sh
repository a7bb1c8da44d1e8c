#!/bin/bash
# Round-3 A/B round trip: parity tests for the changed paths, then the
# c2 encode leg under both settings of an env knob, the E-step leg and the
# BPE-train leg.  Usage (via gpurun): bash tools/gpu_ab.sh TAG KNOB
set -o pipefail
TAG=${1:-ab}
KNOB=${2:-SPM_HIP_ROOT_LDS}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
T="python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread"
env $KNOB=1 timeout -k 10 600 $T $R/tests/test_gpu_parity.py > $O/tests_knob1.log 2>&1 || { echo "TESTS (knob=1) FAILED"; tail -30 $O/tests_knob1.log; exit 1; }
tail -1 $O/tests_knob1.log
timeout -k 10 600 $T $R/tests/test_gpu_estep.py $R/tests/test_gpu_train.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C2="--bpe-steps 0 --raw-steps 0 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --steps 20"
for k in 0 1 0 1; do
  env $KNOB=$k timeout -k 10 300 python3 -u $R/bench.py $C2 > $O/c2_$k.json 2> $O/c2_$k.err || { echo "C2 FAILED"; tail -5 $O/c2_$k.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c2_$k.json')); print('$KNOB=$k', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
ES="--bpe-steps 0 --raw-steps 0 --steps 1 --warmup 1 --sentences 1000000 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 2"
timeout -k 10 400 python3 -u $R/bench.py $ES > $O/estep.json 2> $O/estep.err || { echo "ESTEP FAILED"; tail -5 $O/estep.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/estep.json'))['estep']; print('estep FAST', d['value'], 'PARITY', d['parity']['value'])"
timeout -k 10 400 python3 -u $R/tools/train_bench.py --lines 10000000 --model-type bpe --workers 16 --args "--normalization_rule_name=identity --num_threads=16" > $O/train_bpe_10m.json 2> $O/train_bpe_10m.log || { echo "BPE TRAIN FAILED"; tail -5 $O/train_bpe_10m.log; exit 1; }
cat $O/train_bpe_10m.json
echo DONE
