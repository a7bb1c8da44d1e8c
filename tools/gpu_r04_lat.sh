# Latency leg alone (lib/spm_latency): Encode(single) and encode_batch_host
# over batch sizes.  Usage (via gpurun): bash tools/gpu_r04_lat.sh TAG
set -o pipefail
TAG=${1:-lat}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
python3 -c "import sys; sys.path.insert(0,'$R/tools'); import synth; open('$O/lines.txt','wb').write(b'\n'.join(synth.lines(70000, seed=77)) + b'\n')"
timeout -k 10 300 $R/sentencepiece-comments_amd/lib/spm_latency $R/data/synth32k_unigram.model $O/lines.txt 2000 > $O/latency.json 2> $O/latency.err || { echo LATENCY FAILED; tail -5 $O/latency.err; exit 1; }
cat $O/latency.json
