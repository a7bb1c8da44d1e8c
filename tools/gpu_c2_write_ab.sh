#!/bin/bash
# c2 fast-kernel HBM write traffic (WRITE_SIZE pass) of the in-tree library
# and of variant builds (SPM_AMD_LIB=lib/<var>/libspm_hip.so).
# Usage (via gpurun): bash tools/gpu_c2_write_ab.sh TAG var1 var2 ...
set -o pipefail
TAG=${1:-c2w}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C2="--steps 3 --warmup 1 --bpe-steps 0 --raw-steps 0 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=$R/sentencepiece-comments_amd/lib/$v/libspm_hip.so; fi
  SPM_AMD_LIB=$L timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/w_$v -o run -- python3 $R/bench.py $C2 > $O/w_$v.json 2> $O/w_$v.log || { echo "PMC $v FAILED"; tail -5 $O/w_$v.log; exit 1; }
  SPM_AMD_LIB=$L timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f_$v -o run -- python3 $R/bench.py $C2 > $O/f_$v.json 2> $O/f_$v.log || { echo "PMC $v FAILED"; tail -5 $O/f_$v.log; exit 1; }
  echo "== $v"
  python3 $R/tools/pmc_traffic.py $O/f_$v/run_results.db $O/w_$v/run_results.db "unigram_fast_kernel" $O/pmc_$v.json | grep -E "per_launch|dispatches" -A0
  python3 -c "import json; d=json.load(open('$O/w_$v.json')); print('ms/step', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'])"
done
find $O -name '*.db' -delete
echo DONE
