#!/bin/bash
# Round-6 combined GPU step: cooperative-kernel A/B against a staged library
# (ablib/), every GPU test, then the default bench line.  Stops at the first
# failure; each step has its own time limit.
# Usage (via gpurun): bash tools/gpu_r06_all.sh TAG [AB_TAG]
set -o pipefail
TAG=${1:-r06_all}
AB=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -n "$AB" ]; then
  (AB_OLD=$AB timeout -k 10 200 python3 -u $R/tools/coop_ab.py $AB-a $AB-b && timeout -k 10 200 python3 -u $R/tools/coop_ab.py new-a new-b && AB_OLD=$AB timeout -k 10 200 python3 -u $R/tools/coop_ab.py $AB-c) > $O/coop_ab.txt 2>&1 || { echo "AB FAILED"; tail -5 $O/coop_ab.txt; exit 1; }
  grep -v amdgpu.ids $O/coop_ab.txt
fi
bash $R/tools/gpu_r06.sh $TAG all default
