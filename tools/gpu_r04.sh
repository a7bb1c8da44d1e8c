#!/bin/bash
# Round-4 GPU round trip: all GPU tests, the default bench line, a kernel
# trace of every leg but c5, HBM traffic (FETCH / WRITE passes) and an SQ
# counter pass of the encode kernels.  Summaries land in gpurun_out/TAG/.
# Usage (via gpurun): bash tools/gpu_r03.sh TAG [--no-tests] [bench args...]
set -o pipefail
TAG=${1:-r03}; shift
TESTS=1
if [ "$1" = "--no-tests" ]; then TESTS=0; shift; fi
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
db() { find "$1" -name '*results.db' | head -1; }
if [ $TESTS = 1 ]; then
  timeout -k 10 1200 python3 -u -m pytest $R/tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
timeout -k 10 900 python3 -u $R/bench.py "$@" > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
SHORT="--steps 3 --warmup 1 --bpe-steps 2 --raw-steps 2 --estep-epochs 1 --estep-parity-epochs 1 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $SHORT "$@" > $O/trace.log 2>&1 || { echo "TRACE FAILED"; tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(db $O/trace) $O/kernel_trace.txt > /dev/null
head -30 $O/kernel_trace.txt
C2="--steps 10 --warmup 3 --bpe-steps 0 --raw-steps 0 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run -- python3 $R/bench.py $C2 "$@" > $O/trace_c2.json 2> $O/trace_c2.log || { echo "C2 TRACE FAILED"; tail -5 $O/trace_c2.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(db $O/trace_c2) $O/kernel_trace_c2.txt > /dev/null
head -8 $O/kernel_trace_c2.txt
ENC="--steps 2 --warmup 1 --bpe-steps 2 --raw-steps 0 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 $R/bench.py $ENC "$@" > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 $R/bench.py $ENC "$@" > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -5 $O/pmc_write.log; exit 1; }
python3 $R/tools/pmc_traffic.py $(db $O/pmc_fetch) $(db $O/pmc_write) "unigram_fast_kernel" $O/pmc_unigram_fast.json > /dev/null
python3 $R/tools/pmc_traffic.py $(db $O/pmc_fetch) $(db $O/pmc_write) "bpe_lane_kernel" $O/pmc_bpe_lane.json > /dev/null
cat $O/pmc_unigram_fast.json
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM --kernel-trace -d $O/pmc_sq -o run -- python3 $R/bench.py $ENC "$@" > $O/pmc_sq.log 2>&1 || { echo "PMC SQ FAILED"; tail -5 $O/pmc_sq.log; exit 1; }
python3 $R/tools/sq_counters.py $(db $O/pmc_sq) unigram_fast_kernel > $O/sq_unigram_fast.txt
python3 $R/tools/sq_counters.py $(db $O/pmc_sq) bpe_lane_kernel > $O/sq_bpe_lane.txt
cat $O/sq_unigram_fast.txt $O/sq_bpe_lane.txt
timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_ta -o run -- python3 $R/bench.py $ENC "$@" > $O/pmc_ta.log 2>&1 || { echo "PMC TA FAILED"; tail -5 $O/pmc_ta.log; exit 1; }
python3 $R/tools/sq_counters.py $(db $O/pmc_ta) unigram_fast_kernel > $O/ta_unigram_fast.txt
python3 $R/tools/sq_counters.py $(db $O/pmc_ta) bpe_lane_kernel > $O/ta_bpe_lane.txt
cat $O/ta_unigram_fast.txt $O/ta_bpe_lane.txt
# E-step kernels (PARITY: fold, backward, E-mode forward): SQ + traffic passes.
EST="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check --estep-sentences 12500000 --estep-epochs 1 --estep-warmup 0 --estep-parity-epochs 1"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM --kernel-trace -d $O/pmc_sq_estep -o run -- python3 $R/bench.py $EST "$@" > $O/pmc_sq_estep.log 2>&1 || { echo "PMC SQ ESTEP FAILED"; tail -5 $O/pmc_sq_estep.log; exit 1; }
for k in "estep_fold_kernel" "estep_backward_kernel<16, 4, 10>" "estep_backward_kernel<16, 3, 8>" "unigram_fast_kernel<16, true, 4, true>" "estep_compact_records"; do echo "== $k"; python3 $R/tools/sq_counters.py $O/pmc_sq_estep/run_results.db "$k"; done > $O/sq_estep.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch_estep -o run -- python3 $R/bench.py $EST "$@" > $O/pmc_fetch_estep.log 2>&1 || { echo "PMC FETCH ESTEP FAILED"; tail -5 $O/pmc_fetch_estep.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write_estep -o run -- python3 $R/bench.py $EST "$@" > $O/pmc_write_estep.log 2>&1 || { echo "PMC WRITE ESTEP FAILED"; tail -5 $O/pmc_write_estep.log; exit 1; }
for k in "estep_fold_kernel" "estep_backward_kernel<16, 4, 10>" "unigram_fast_kernel<16, true, 4, true>"; do python3 $R/tools/pmc_traffic.py $O/pmc_fetch_estep/run_results.db $O/pmc_write_estep/run_results.db "$k" $O/pmc_estep_$(echo $k | tr -cd 'a-z0-9_').json > /dev/null; done
cat $O/sq_estep.txt
find $O -name '*.db' -delete
echo DONE
