#!/bin/bash
# Per-call latency phases (SPM_HIP_SERVICE_PROF) of lib/spm_latency on botchan
# + test_model.model, optionally GPU tests first, and the cooperative list
# kernel A/B against ablib/<OLD> (tools/coop_ab.py) to check the batch path.
# Usage (via gpurun): bash tools/gpu_r06_lat.sh TAG [OLD_TAG] ["TESTS"]
set -o pipefail
TAG=${1:-r06_lat}
OLD=${2:-}
TESTS=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  (cd $R && timeout -k 10 600 python3 -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread) > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -30; tail -20 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
SPM_HIP_SERVICE_PROF=1 timeout -k 10 120 $R/sentencepiece-comments_amd/lib/spm_latency $R/tests/golden/test_model.model $R/tests/golden/botchan.txt 4288 > $O/lat.json 2> $O/lat.err || { echo "LATENCY FAILED"; tail -5 $O/lat.err; exit 1; }
grep "raw call prof" $O/lat.err
python3 -c "import json; d=json.load(open('$O/lat.json')); print('encode_single_us', d['encode_single_us'], 'batch1', d['batches'][0]['us_per_call'])"
if [ -n "$OLD" ]; then
  for i in 1 2; do
    timeout -k 10 200 python3 $R/tools/coop_ab.py slab=0 2>&1 | grep -v amdgpu.ids | sed 's/^/new /' >> $O/ab.txt || exit 1
    AB_OLD=$OLD timeout -k 10 200 python3 $R/tools/coop_ab.py slab=0 2>&1 | grep -v amdgpu.ids | sed 's/^/old /' >> $O/ab.txt || exit 1
  done
  cat $O/ab.txt
fi
