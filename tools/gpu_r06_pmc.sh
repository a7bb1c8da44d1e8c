#!/bin/bash
# Stamped PMC summaries of the shipped kernels for bench.py (profiles/pmc/):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (MI355X_MICROARCH.md
# HBM section), per bench leg: c2 + c3 (one run), the Japanese leg (lane
# kernel + cooperative kernel) and the c4 PARITY E-step pipeline.  Each
# summary carries the kernel sources' sha256, so bench.py reports it only
# for these very kernels.
# Usage (via gpurun): bash tools/gpu_r06_pmc.sh TAG COMMIT [LEGS]
set -o pipefail
TAG=${1:-r06_pmc}
COMMIT=${2:-unknown}
LEGS=${3:-"enc ja c4"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O $O/pmc
cd /tmp && export TMPDIR=/tmp
# The PMC databases stay on the box whatever happens (gpurun copies back at most 64 MiB).
trap 'find $O -name "*.db" -delete' EXIT
OFF="--raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
pass() {  # name counter args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d $O/$name -o run -- python3 $R/bench.py "$@" --detail $O/$name.detail.json > $O/$name.log 2>&1 || { echo "PMC $name FAILED"; tail -5 $O/$name.log; exit 1; }
  find $O/$name -name '*results.db' | head -1
}
for leg in $LEGS; do
  case $leg in
    enc)
      A="--steps 2 --warmup 1 --sentences 10000000 --bpe-steps 2 --ja-lines 0 --estep-sentences 0 $OFF"
      F=$(pass enc_fetch FETCH_SIZE $A) || exit 1
      W=$(pass enc_write WRITE_SIZE $A) || exit 1
      python3 $R/tools/pmc_traffic.py $F $W c2 $O/pmc unigram_fast_kernel --commit $COMMIT --units 10000000 || exit 1
      python3 $R/tools/pmc_traffic.py $F $W c3 $O/pmc bpe_lane_kernel bpe_fast_kernel bpe_compact_kernel --commit $COMMIT --units 10000000 || exit 1
      python3 $R/tools/kernel_names.py $F > $O/enc_kernels.txt ;;
    ja)
      A="--steps 1 --warmup 1 --sentences 100000 --bpe-steps 0 --estep-sentences 0 $OFF"
      F=$(pass ja_fetch FETCH_SIZE $A) || exit 1
      W=$(pass ja_write WRITE_SIZE $A) || exit 1
      python3 $R/tools/pmc_traffic.py $F $W ja $O/pmc "unigram_fast_kernel<16, false, 3" --commit $COMMIT || exit 1
      python3 $R/tools/pmc_traffic.py $F $W ja_coop $O/pmc coop_list_kernel --commit $COMMIT || exit 1
      python3 $R/tools/kernel_names.py $F > $O/ja_kernels.txt ;;
    c4)
      # One warm-up + one timed PARITY epoch of 50 M sentences (chunks as the
      # bench's: a small first chunk, then up to 6.25 M): traffic per
      # sentence = all dispatches' bytes / all sentences.
      A="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --ja-lines 0 --estep-sentences 50000000 --estep-parity-epochs 1 --estep-warmup 1 $OFF"
      F=$(pass c4_fetch FETCH_SIZE $A) || exit 1
      W=$(pass c4_write WRITE_SIZE $A) || exit 1
      python3 $R/tools/pmc_traffic.py $F $W c4 $O/pmc "unigram_fast_kernel<16, true, 4, true" estep_backward_kernel estep_compact_records_kernel estep_fold_kernel --commit $COMMIT --units-total 150000000 || exit 1
      python3 $R/tools/kernel_names.py $F > $O/c4_kernels.txt ;;
  esac
done
find $O -name '*.db' -delete
echo DONE
