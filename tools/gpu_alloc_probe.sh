#!/bin/bash
# Where does hipMalloc start to wait right after another process freed 200 / 160 GiB?
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05an; mkdir -p $O; cd /tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 $R/tools/alloc_probe.cc -o /tmp/alloc_probe || exit 1
fill() { timeout -k 10 120 python3 -c "
import torch
xs = [torch.ones(1 << 30, dtype=torch.uint8, device='cuda') for _ in range($1)]
torch.cuda.synchronize(); print('filled', len(xs))
"; }
{ fill 200 && timeout -k 10 60 /tmp/alloc_probe 120 4 && sleep 20 && fill 160 && timeout -k 10 60 /tmp/alloc_probe 120 4; } > $O/probe.txt 2>&1
grep -v amdgpu.ids $O/probe.txt
