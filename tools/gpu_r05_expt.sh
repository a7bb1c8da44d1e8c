#!/bin/bash
# E-step traffic attribution (temporary knob SPM_HIP_ESTEP_EXPT): bit 1 = the
# backward pass reads no alpha, bit 2 = the forward pass writes no alpha,
# bit 4 = the backward pass stores no records.  Per value: kernel times from
# the bench and FETCH / WRITE per launch of both passes.
set -o pipefail
TAG=${1:-r05_expt}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ES="--bpe-steps 0 --raw-steps 0 --steps 1 --warmup 1 --sentences 100000 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 1 --estep-parity-epochs 2 --ja-lines 0 --latency-calls 0 --no-parity-check"
EST="--steps 1 --warmup 0 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check --estep-sentences 12500000 --estep-epochs 1 --estep-warmup 0 --estep-parity-epochs 1"
for v in "$@"; do
  export SPM_HIP_ESTEP_EXPT=$v
  timeout -k 10 300 python3 -u $R/bench.py $ES > $O/estep_$v.json 2> $O/estep_$v.err || { echo "ESTEP $v FAILED"; tail -5 $O/estep_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/estep_$v.json'))['estep']; r=d['parity']['roofline']; print('EXPT=$v PARITY', round(d['parity']['value'],4), 'fwd_ms', round(r['forward_kernel_ms'],3), 'bwd_ms', round(r['kernel_ms'],3))"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f$v -o run -- python3 $R/bench.py $EST > $O/f$v.log 2>&1 || { echo "PMC FETCH FAILED"; tail -5 $O/f$v.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/w$v -o run -- python3 $R/bench.py $EST > $O/w$v.log 2>&1 || { echo "PMC WRITE FAILED"; tail -5 $O/w$v.log; exit 1; }
  for k in "estep_backward_kernel<16, 4, 10>" "unigram_fast_kernel<16, true, 4, true"; do
    python3 $R/tools/pmc_traffic.py $(find $O/f$v -name '*results.db' | head -1) $(find $O/w$v -name '*results.db' | head -1) "$k" $O/pmc_${v}_$(echo $k | tr -cd 'a-z0-9_').json > /dev/null
    python3 -c "import json; d=json.load(open('$O/pmc_${v}_$(echo $k | tr -cd 'a-z0-9_').json')); t=sorted(a+b for a,b in zip(d['read_bytes_per_dispatch'], d['write_bytes_per_dispatch'])); print('  $k read %.2f write %.2f GB/launch (mean), median total %.2f' % (d['hbm_read_bytes_per_launch']/1e9, d['hbm_write_bytes_per_launch']/1e9, t[len(t)//2]/1e9))"
  done
  find $O -name '*.db' -delete
done
echo DONE
