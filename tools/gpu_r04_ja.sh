# Multi-byte (ja) leg alone + its SQ/TA counters.  Usage: bash tools/gpu_r04_ja.sh TAG
set -o pipefail
TAG=${1:-ja}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
JA="--steps 3 --warmup 1 --bpe-steps 0 --raw-steps 0 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --sentences 100000"
timeout -k 10 300 python3 $R/bench.py $JA > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); j=d['ja_multibyte']; print(j['value'], j['roofline']['kernel'], j['roofline']['kernel_ms'], d['parity']['ja_multibyte']['mismatches'])"
JB="$JA --no-parity-check --steps 1 --warmup 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-trace -d $O/pmc_sq -o run -- python3 $R/bench.py $JB > $O/pmc_sq.log 2>&1 || { echo "PMC SQ FAILED"; tail -5 $O/pmc_sq.log; exit 1; }
python3 $R/tools/sq_counters.py $O/pmc_sq/run_results.db "false, 3, false, true>" > $O/sq_wide.txt
timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_ta -o run -- python3 $R/bench.py $JB > $O/pmc_ta.log 2>&1 || { echo "PMC TA FAILED"; tail -5 $O/pmc_ta.log; exit 1; }
python3 $R/tools/sq_counters.py $O/pmc_ta/run_results.db "false, 3, false, true" > $O/ta_wide.txt
cat $O/sq_wide.txt $O/ta_wide.txt
