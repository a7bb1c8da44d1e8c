#!/bin/bash
# PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the cooperative
# kernel on the Japanese leg (bench.py default --ja-lines), then the leg
# itself with the committed summary in its roofline.coop object.
set -o pipefail
TAG=${1:-r05_ja_pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
JA="--steps 1 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run -- python3 $R/bench.py $JA > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run -- python3 $R/bench.py $JA > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail -5 $O/pmc_write.log; exit 1; }
python3 $R/tools/pmc_traffic.py $(find $O/pmc_fetch -name '*results.db' | head -1) $(find $O/pmc_write -name '*results.db' | head -1) "coop_list_kernel" $O/pmc_ja_coop.json > $O/pmc.txt 2>&1 || { echo "PMC SUMMARY FAILED"; tail -5 $O/pmc.txt; exit 1; }
grep -E "hbm_|dispatches" -A2 $O/pmc.txt | head -12
cp $O/pmc_ja_coop.json $R/profiles/r05_pmc_ja_coop.json
JA2="--steps 3 --warmup 1 --sentences 100000 --bpe-steps 0 --raw-steps 0 --train-lines 0 --bpe-train-lines 0 --latency-calls 0 --estep-sentences 0 --no-cpu-baseline --no-probe-stats"
timeout -k 10 400 python3 -u $R/bench.py $JA2 > $O/ja.json 2> $O/ja.err || { echo "JA FAILED"; tail -5 $O/ja.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ja.json')); j=d['ja_multibyte']; print('ja', round(j['value']/1e6,2), 'M/s', json.dumps(j['roofline'].get('coop')), d.get('parity',{}).get('ja_multibyte',{}).get('mismatches'))"
find $O -name '*.db' -delete
echo DONE
