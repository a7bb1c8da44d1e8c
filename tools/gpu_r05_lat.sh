#!/bin/bash
# Round-5 latency check: small-batch / async / parity GPU tests, then the
# per-call latency tool on botchan (c1) with the 32k synthetic model too.
set -o pipefail
TAG=${1:-r05_lat}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $R/tests/test_gpu_small_batch.py $R/tests/test_gpu_async.py $R/tests/test_gpu_parity.py $R/tests/test_gpu_concurrency.py $R/tests/test_gpu_cli.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 $R/sentencepiece-comments_amd/lib/spm_latency $R/tests/golden/test_model.model $R/tests/golden/botchan.txt 3000 > $O/latency_botchan.json 2> $O/latency.err || { cat $O/latency.err; exit 1; }
cat $O/latency_botchan.json
