# Short GPU round trip after a kernel change: encode / E-step / train / async
# GPU tests, then the c2 + c4 bench legs (no CPU baselines, no c5) and a
# kernel trace of the same run.
# Usage (via gpurun): bash tools/gpu_ab_short.sh TAG
set -o pipefail
TAG=${1:-short}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_estep.py $R/tests/test_gpu_train.py $R/tests/test_gpu_async.py $R/tests/test_gpu_dist_estep.py $R/tests/test_gpu_cli.py $R/tests/test_gpu_concurrency.py $R/tests/test_gpu_spt.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
B="--steps 10 --warmup 3 --bpe-steps 5 --raw-steps 3 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 2 --estep-parity-epochs 2"
timeout -k 10 400 python3 $R/bench.py $B > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); e=d['estep']
b=d['bpe_c3']; print('c2 %.4g sent/s kernel %.3f ms step %.3f ms | c3 %.4g sent/s kernel %.3f ms | e2e %.4g | c4 FAST %.4f PARITY %.4f s/epoch obj %r %r' % (d['value'], d['roofline']['kernel_ms'], d['ms_per_step'], b['value'], b['roofline']['kernel_ms'], d['e2e_raw']['value'], e['value'], e['parity']['value'], e['obj'], e['parity']['obj']))"
S="--steps 3 --warmup 1 --bpe-steps 2 --raw-steps 2 --train-lines 0 --bpe-train-lines 0 --no-cpu-baseline --no-probe-stats --estep-epochs 1 --estep-parity-epochs 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py $S > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace.txt | head -16
