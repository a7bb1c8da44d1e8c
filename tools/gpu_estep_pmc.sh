# SQ counters of the c4 E-step FAST kernels (one rocprofv3 --pmc pass).
set -o pipefail
TAG=${1:-estep_pmc}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 1 --estep-warmup 0 --estep-parity-epochs 0 --estep-sentences 12500000"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-trace -d $O/pmc -o run -- python3 $R/bench.py $ARGS > $O/bench.json 2> $O/pmc.log || { echo PMC FAILED; tail -5 $O/pmc.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES --kernel-trace -d $O/pmc2 -o run -- python3 $R/bench.py $ARGS > $O/bench2.json 2> $O/pmc2.log || { echo PMC2 FAILED; tail -5 $O/pmc2.log; }
for k in estep_forward estep_backward; do echo "== $k"; python3 $R/tools/sq_counters.py $O/pmc/run_results.db $k; python3 $R/tools/sq_counters.py $O/pmc2/run_results.db $k 2>/dev/null; done
echo DONE
