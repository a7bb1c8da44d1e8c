#!/bin/bash
# Round-4 check: every GPU test, the default bench line, then (optional
# steps, each under its own time limit) the device corpus load at 10 M lines
# and the c2 write A/B.  Usage (via gpurun): bash tools/gpu_r04_final.sh TAG
set -o pipefail
TAG=${1:-r04final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest $R/tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("c2", d["value"], "kernel_ms", d["roofline"]["kernel_ms"])
for k in ("bpe_c3", "estep", "train", "multibyte", "parity"):
    v = d.get(k)
    if isinstance(v, dict):
        print(k, {x: v.get(x) for x in ("value", "unit", "mismatches") if x in v}, (v.get("parity") or {}).get("value") if k == "estep" else "")
PY
echo DONE
