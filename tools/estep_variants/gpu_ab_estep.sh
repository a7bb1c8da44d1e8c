# E-step A/B round trip: E-step/train tests (walk-once default), then the c4
# leg with the walk-once kernels and with the two-walk kernels.
# Usage (via gpurun): bash tools/gpu_ab_estep.sh TAG
set -o pipefail
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_estep.py $R/tests/test_gpu_dist_estep.py $R/tests/test_gpu_train.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_async.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
ES="--steps 2 --warmup 1 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 2"
for l in 1 0; do
  SPM_HIP_ESTEP_LIST=$l timeout -k 10 300 python3 $R/bench.py $ES > $O/es_$l.json 2> $O/es_$l.err || { tail -5 $O/es_$l.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/es_$l.json'))['estep']; print('list $l FAST %.4f s/epoch PARITY %.4f s/epoch' % (d['value'], d['parity']['value']), d['ntok'], d['obj'], d['parity']['obj'])"
done
SPM_HIP_ESTEP_LIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $ES > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace.txt | head -16
