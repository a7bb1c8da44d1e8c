#!/bin/bash
# A/B of the cooperative kernel against another build's library (ablib/,
# AB_OLD tag) on the Japanese corpus: tools/coop_ab.py, alternating, then one
# SPM_HIP_COOP_PROF pass each (phase cycles).  Optional first: GPU tests.
# Usage (via gpurun): bash tools/gpu_r06_ab.sh TAG OLD_TAG ["TESTS"]
set -o pipefail
TAG=${1:-r06_ab}
OLD=${2:-r06m}
TESTS=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  (cd $R && timeout -k 10 600 python3 -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread) > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -30; tail -20 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
for i in 1 2; do
  timeout -k 10 200 python3 $R/tools/coop_ab.py slab=0 2>&1 | grep -v amdgpu.ids | sed 's/^/new /' >> $O/ab.txt || exit 1
  AB_OLD=$OLD timeout -k 10 200 python3 $R/tools/coop_ab.py slab=0 2>&1 | grep -v amdgpu.ids | sed 's/^/old /' >> $O/ab.txt || exit 1
done
SPM_HIP_COOP_PROF=1 timeout -k 10 200 python3 $R/tools/coop_ab.py slab=0 2>&1 | grep -v amdgpu.ids | tail -2 | sed 's/^/new /' >> $O/ab.txt || exit 1
SPM_HIP_COOP_PROF=1 AB_OLD=$OLD timeout -k 10 200 python3 $R/tools/coop_ab.py slab=0 2>&1 | grep -v amdgpu.ids | tail -2 | sed 's/^/old /' >> $O/ab.txt || exit 1
cat $O/ab.txt
