#!/bin/bash
# A/B of SPM_HIP_ESTEP_WPE on the c4 E-step bench leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/wpe
cd /tmp
for w in 2 3 4; do
  SPM_HIP_ESTEP_WPE=$w timeout -k 10 200 python3 $R/bench.py --steps 1 --warmup 1 --raw-steps 0 --train-lines 0 --no-cpu-baseline > $R/gpurun_out/wpe/b$w.json 2> $R/gpurun_out/wpe/e$w.txt || { tail -5 $R/gpurun_out/wpe/e$w.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$R/gpurun_out/wpe/b$w.json'));print('wpe $w', d['estep']['value'])"
done
