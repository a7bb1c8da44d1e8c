#!/bin/bash
# Latency A/B on one box: latency building blocks, then spm_latency on botchan
# under SPM_HIP_SMALL_ZEROCOPY = 0 / 1 / 0 / 1.
set -o pipefail
TAG=${1:-r05_lat_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/sentencepiece-comments_amd/lib/latency_probe 3000 > $O/latency_probe.txt 2>&1 || { cat $O/latency_probe.txt; exit 1; }
cat $O/latency_probe.txt
for v in 0 1 0 1; do
  SPM_HIP_SMALL_ZEROCOPY=$v timeout -k 10 120 $R/sentencepiece-comments_amd/lib/spm_latency $R/tests/golden/test_model.model $R/tests/golden/botchan.txt 3000 > $O/lat_$v.json 2> $O/lat.err || { cat $O/lat.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lat_$v.json')); print('zerocopy=$v', 'single', d['encode_single_us'], [(b['batch'], round(b['us_per_call'],1)) for b in d['batches']])"
done
