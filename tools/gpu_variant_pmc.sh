#!/bin/bash
# Unigram fast-kernel variant A/B (time) + per-variant HBM traffic (PMC passes).
# Usage (via gpurun): bash tools/gpu_variant_pmc.sh TAG VARIANTS
set -o pipefail
TAG=$1; V=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
M=$R/data/synth32k_unigram.model
timeout -k 10 300 python3 $R/tools/variant_bench.py 10000000 $M $V > $O/variant_ab.txt 2>&1 || { tail -5 $O/variant_ab.txt; exit 1; }
grep variant $O/variant_ab.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 $R/tools/variant_bench.py 2000000 $M $V > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 $R/tools/variant_bench.py 2000000 $M $V > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; exit 1; }
echo DONE
