# Quick GPU round trip: selected tests (args) -> gpurun_out/quick/tests.log
set -o pipefail
mkdir -p gpurun_out/quick
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > $R/gpurun_out/quick/tests.log 2>&1 || { tail -60 $R/gpurun_out/quick/tests.log; exit 1; }
tail -3 $R/gpurun_out/quick/tests.log
