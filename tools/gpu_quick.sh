# Quick GPU round trip: selected tests (args, paths relative to the repo root
# or pytest options) -> gpurun_out/${QTAG:-quick}/tests.log
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${QTAG:-quick}
mkdir -p $O
args=()
for a in "$@"; do
  case $a in tests/*) a=$R/$a ;; esac
  args+=("$a")
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest "${args[@]}" -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
