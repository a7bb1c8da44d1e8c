# c3 A/B of bpe_lane_kernel<true> (rank ids, 17.5 KB LDS) vs <false>
# (32-bit symbol words, 25.5 KB), alternating, c3 leg only.
# Usage (via gpurun): bash tools/gpu_r04_bpe_ab.sh TAG
set -o pipefail
TAG=${1:-bpe_ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 1 --warmup 1 --bpe-steps 10 --raw-steps 0 --estep-sentences 0 --train-lines 0 --bpe-train-lines 0 --ja-lines 0 --latency-calls 0 --no-cpu-baseline --no-probe-stats --no-parity-check"
for k in 1 0 1 0; do
  SPM_HIP_BPE_RANK_IDS=$k timeout -k 10 300 python3 $R/bench.py $ARGS > $O/ab_$k.json 2> $O/ab_$k.err || { echo "AB $k FAILED"; tail -5 $O/ab_$k.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/ab_$k.json'))['bpe_c3']; print('rank_ids=$k', d['value'], d['roofline']['kernel_ms'])" | tee -a $O/ab.txt
done
