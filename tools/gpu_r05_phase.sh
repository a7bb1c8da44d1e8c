#!/bin/bash
# Cooperative kernel phase cycles, one sentence per launch (latency case).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r05ar_phase}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
SPM_HIP_COOP_PROF=1 timeout -k 10 300 python3 -u $R/tools/coop_phase_latency.py > $O/out.txt 2> $O/prof.txt || { echo FAILED; tail -5 $O/prof.txt; exit 1; }
cat $O/out.txt
grep "coop prof" $O/prof.txt | awk '{for(i=1;i<=NF;i++){if($i=="setup")a+=$(i+1);if($i=="lattice")b+=$(i+1);if($i=="viterbi")c+=$(i+1);if($i=="backtrace")d+=$(i+1);if($i=="ids")e+=$(i+1);if($i=="bytes")f+=$(i+1);if($i=="tokens")g+=$(i+1)}} END {print "calls",NR,"setup",a/NR,"lattice",b/NR,"viterbi",c/NR,"backtrace",d/NR,"ids",e/NR,"bytes",f/NR,"tokens",g/NR, "cycles/byte viterbi", c/f, "lattice", b/f, "cycles/token backtrace", d/g}'
