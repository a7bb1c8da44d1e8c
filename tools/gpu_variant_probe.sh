#!/bin/bash
# Per-variant golden-corpus probe, one process per case, each under a timeout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
M=tests/golden/test_model.model; T=tests/golden/botchan.txt
for v in ${1:-115960 247032}; do
  echo "== $v"
  timeout -k 5 60 python3 -u $R/tools/variant_probe.py $v $M $T || { echo "FAILED rc=$?"; exit 1; }
done
echo DONE
