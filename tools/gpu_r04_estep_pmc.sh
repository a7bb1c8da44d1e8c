#!/bin/bash
# E-step counters: one c4 PARITY + FAST epoch at 12.5 M
# sentences under separate rocprofv3 --pmc passes (SQ, TA, FETCH, WRITE).
# Usage (via gpurun): bash tools/gpu_r04_estep_pmc.sh TAG
set -o pipefail
TAG=${1:-r04_estep_pmc}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
EST="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check --estep-sentences 12500000 --estep-epochs 1 --estep-warmup 0 --estep-parity-epochs 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $EST > $O/trace.json 2> $O/trace.log || { echo "TRACE FAILED"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $O/trace/run_results.db $O/kernel_trace.txt > /dev/null
head -24 $O/kernel_trace.txt
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM --kernel-trace -d $O/pmc_sq -o run -- python3 $R/bench.py $EST > $O/pmc_sq.log 2>&1 || { echo "PMC SQ FAILED"; tail -5 $O/pmc_sq.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_ta -o run -- python3 $R/bench.py $EST > $O/pmc_ta.log 2>&1 || { echo "PMC TA FAILED"; tail -5 $O/pmc_ta.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 $R/bench.py $EST > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 $R/bench.py $EST > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -5 $O/pmc_write.log; exit 1; }
for k in "estep_fold_kernel" "estep_backward_kernel<16, 4, 10>" "estep_backward_kernel<16, 3, 8>" "unigram_fast_kernel<16, true, 4, true>" "estep_compact_records" "estep_threshold"; do
  echo "== $k"
  python3 $R/tools/sq_counters.py $O/pmc_sq/run_results.db "$k"
  python3 $R/tools/sq_counters.py $O/pmc_ta/run_results.db "$k"
  python3 $R/tools/pmc_traffic.py $O/pmc_fetch/run_results.db $O/pmc_write/run_results.db "$k" $O/pmc_$(echo $k | tr -cd 'a-z0-9_').json
done > $O/estep_counters.txt 2>&1
cat $O/estep_counters.txt
# (the result databases are large: keep only the text summaries)
find $O -name '*.db' -delete
find $O -name '*.csv' -delete
echo DONE
