# c2 A/B round trip: encode tests (under each output scheme), then the c2 leg
# alone under each setting.  Usage (via gpurun): bash tools/gpu_ab_c2.sh TAG
set -o pipefail
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for out in dense slot; do
  SPM_HIP_ENCODE_OUT=$out timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_async.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_$out.log 2>&1 || { tail -30 $O/tests_$out.log; exit 1; }
  echo "tests ($out): $(tail -1 $O/tests_$out.log)"
done
C2="--steps 20 --warmup 3 --bpe-steps 0 --raw-steps 3 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats"
for out in dense slot dense slot; do
  SPM_HIP_ENCODE_OUT=$out timeout -k 10 300 python3 $R/bench.py $C2 > $O/c2_$out.json 2> $O/c2_$out.err || { tail -5 $O/c2_$out.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c2_$out.json')); print('$out', d['value']/1e9, 'G/s', d['ms_per_step'], 'ms/step kernel', d['roofline']['kernel_ms'], 'e2e', d['e2e_raw']['ms_per_step'])"
done
SPM_HIP_ENCODE_OUT=slot timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $C2 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace.txt | head -16
