#!/bin/bash
# Round-5 E-step check: E-step GPU tests, c4 A/B of an env knob (alternating),
# then PMC traffic (FETCH_SIZE / WRITE_SIZE / TCC hit-miss) of the PARITY
# backward kernel under the knob's last value.
# Usage (via gpurun): bash tools/gpu_r05_estep.sh TAG KNOB v1 v2 ...
set -o pipefail
TAG=${1:-r05_estep}; KNOB=${2:-SPM_HIP_ESTEP_STAGE}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_estep.py $R/tests/test_gpu_train.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ES="--bpe-steps 0 --raw-steps 0 --steps 1 --warmup 1 --sentences 1000000 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 2 --ja-lines 0 --latency-calls 0 --no-parity-check"
last=""
for v in "$@"; do
  env $KNOB=$v timeout -k 10 400 python3 -u $R/bench.py $ES > $O/estep_$v.json 2> $O/estep_$v.err || { echo "ESTEP FAILED"; tail -5 $O/estep_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/estep_$v.json'))['estep']; print('$KNOB=$v FAST', d['fast']['value'], 'PARITY', d['parity']['value'], 'bwd_ms', (d['parity'].get('roofline') or {}).get('kernel_ms'))"
  last=$v
done
EST="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check --estep-sentences 12500000 --estep-epochs 1 --estep-warmup 0 --estep-parity-epochs 1"
export $KNOB=$last
# Equal 6.25 M-sentence chunks in the PMC passes (the units each steady dispatch holds).
export SPM_HIP_ESTEP_FIRST=0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 $R/bench.py $EST > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 $R/bench.py $EST > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -5 $O/pmc_write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TA_BUSY_avr --kernel-trace -d $O/pmc_tcc -o run -- python3 $R/bench.py $EST > $O/pmc_tcc.log 2>&1 || { echo "PMC TCC FAILED"; tail -5 $O/pmc_tcc.log; exit 1; }
for k in "estep_backward_kernel<16, 4, 42>" "estep_backward_kernel<16, 4, 10>" "estep_backward_kernel<16, 3, 40>" "estep_backward_kernel<16, 3, 8>" "unigram_fast_kernel<16, true, 4, true" "estep_compact_records" "estep_fold_kernel"; do
  echo "== $k"
  python3 $R/tools/sq_counters.py $(find $O/pmc_tcc -name '*results.db' | head -1) "$k"
  python3 $R/tools/pmc_traffic.py $(find $O/pmc_fetch -name '*results.db' | head -1) $(find $O/pmc_write -name '*results.db' | head -1) "$k" $O/pmc_$(echo $k | tr -cd 'a-z0-9_').json 6250000
done > $O/estep_counters.txt 2>&1
grep -E "==|hbm_|TCC|dispatches" $O/estep_counters.txt || true
find $O -name '*.db' -delete
echo DONE
