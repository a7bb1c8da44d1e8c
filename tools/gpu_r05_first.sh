#!/bin/bash
# Round-5 first box check: latency building blocks, then the GPU test suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/sentencepiece-comments_amd/lib/latency_probe 3000 > $O/latency_probe.txt 2>&1 || { cat $O/latency_probe.txt; exit 1; }
cat $O/latency_probe.txt
timeout -k 10 900 python3 -u -m pytest $R/tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
