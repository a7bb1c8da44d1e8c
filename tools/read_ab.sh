set -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 200 python3 -c "
import sys; sys.path.insert(0,'tools'); import train_bench as tb; tb.write_corpus('/tmp/c5_corpus.txt', 100000000, 1234, workers=16)
" > gpurun_out/r03w/gen.log 2>&1 || { tail -5 gpurun_out/r03w/gen.log; exit 1; }
timeout -k 10 200 tools/bin/read_ab /tmp/c5_corpus.txt > gpurun_out/r03w/read_ab.txt 2>&1
timeout -k 10 200 tools/bin/read_ab /tmp/c5_corpus.txt >> gpurun_out/r03w/read_ab.txt 2>&1
cat gpurun_out/r03w/read_ab.txt
rm -f /tmp/c5_corpus.txt
