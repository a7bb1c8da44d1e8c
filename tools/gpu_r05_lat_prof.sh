#!/bin/bash
# Where a batch-1 encode call's time goes: kernel durations of spm_latency
# under rocprofv3 (kernel trace), and the GPU clocks around it.
set -o pipefail
TAG=${1:-r05_lat_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
(rocm-smi --showclocks 2>&1 | head -30) > $O/clocks_before.txt || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- $R/sentencepiece-comments_amd/lib/spm_latency $R/tests/golden/test_model.model $R/tests/golden/botchan.txt 1000 > $O/lat_traced.json 2> $O/trace.log || { tail -5 $O/trace.log; exit 1; }
(rocm-smi --showclocks 2>&1 | head -30) > $O/clocks_after.txt || true
python3 $R/tools/rocprof_summary.py $(find $O/trace -name '*results.db' | head -1) $O/kernel_trace.txt > /dev/null
head -20 $O/kernel_trace.txt
python3 $R/tools/rocprof_timeline.py $(find $O/trace -name '*results.db' | head -1) 2>/dev/null | head -5 || true
find $O -name '*.db' -delete
grep -i "sclk\|mclk" $O/clocks_before.txt | head -4
