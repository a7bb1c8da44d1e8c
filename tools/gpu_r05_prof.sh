#!/bin/bash
# E-step PARITY epoch kernel trace (per-kernel stats, GPU busy fraction), SQ
# counters of the E-step and BPE lane kernels.
set -o pipefail
TAG=${1:-r05_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
EST="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check --estep-epochs 1 --estep-warmup 0 --estep-parity-epochs 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $EST > $O/trace.json 2> $O/trace.log || { echo "TRACE FAILED"; tail -5 $O/trace.log; exit 1; }
DB=$(find $O/trace -name '*results.db' | head -1)
python3 $R/tools/rocprof_summary.py $DB $O/estep_kernel_trace.txt > /dev/null
head -24 $O/estep_kernel_trace.txt
python3 $R/tools/trace_busy.py $DB estep_backward_kernel estep_finalize > $O/estep_busy.txt 2>&1; cat $O/estep_busy.txt
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-trace -d $O/sq -o run -- python3 $R/bench.py $EST > $O/sq.log 2>&1 || { echo "SQ FAILED"; tail -5 $O/sq.log; exit 1; }
for k in "estep_backward_kernel<16, 4, 42>" "unigram_fast_kernel<16, true, 4, true" "estep_compact_records" "estep_fold_kernel"; do echo "== $k"; python3 $R/tools/sq_counters.py $(find $O/sq -name '*results.db' | head -1) "$k"; done > $O/sq_estep.txt 2>&1; cat $O/sq_estep.txt
P3="--steps 2 --warmup 1 --sentences 10000000 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --ja-lines 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-trace -d $O/sqb -o run -- python3 $R/bench.py $P3 > $O/sqb.log 2>&1 || { echo "SQB FAILED"; tail -5 $O/sqb.log; exit 1; }
for k in "bpe_lane_kernel" "bpe_fast_kernel" "unigram_fast_kernel<16, true, 7"; do echo "== $k"; python3 $R/tools/sq_counters.py $(find $O/sqb -name '*results.db' | head -1) "$k"; done > $O/sq_encode.txt 2>&1; cat $O/sq_encode.txt
find $O -name '*.db' -delete
echo DONE
