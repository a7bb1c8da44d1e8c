#!/bin/bash
# Where the per-line Encode time goes on real text: the raw latency probe
# alone, then under a kernel trace (per-kernel durations).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r05ao_lat}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/tools/raw_latency_probe.py > $O/probe.txt 2>&1 || { echo PROBE FAILED; tail -5 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/tools/raw_latency_probe.py > $O/probe_kt.txt 2>&1 || { echo KT FAILED; tail -5 $O/probe_kt.txt; exit 1; }
f=$(find $O/kt -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 $f | head -12
