#!/bin/bash
# Per-kernel VGPR / spill / LDS / occupancy report of one HIP source (clang's
# kernel-resource-usage remarks).  Usage: tools/kernel_resources.sh csrc/FILE.hip [kernel-substring]
S=${1:?source}; K=${2:-}
cd "$(dirname "$0")/../sentencepiece-comments_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I csrc --offload-arch=gfx950 -munsafe-fp-atomics \
  --cuda-device-only -Rpass-analysis=kernel-resource-usage -c "$S" -o /tmp/kres_$$.o 2>&1 |
  grep -E "remark: (Function Name|[[:space:]]*(VGPRs|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs Spill|VGPRs Spill))" |
  sed -e 's/.*remark: //' | awk -v k="$K" '/Function Name/{show = (k == "" || index($0, k) > 0)} show'
rm -f /tmp/kres_$$.o
