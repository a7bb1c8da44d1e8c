"""A/B the unigram fast-kernel variants in one process (tuning tool).
Checks every variant's output equals variant 0's and prints fast-kernel ms."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sentencepiece-comments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch
import spm_amd
import synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
model = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "data", "synth32k_unigram.model")
variants = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else list(range(8))
dev = torch.device("cuda", 0)
buf, off = synth.normalized(n, seed=1234)
d_b = torch.from_numpy(buf).to(dev)
d_o = torch.from_numpy(off.view(np.int64)).to(dev)
d_i = torch.empty(int(off[-1]), dtype=torch.int32, device=dev)
d_t = torch.empty(n + 1, dtype=torch.int64, device=dev)
mb = open(model, "rb").read()
ref = None
for rep in range(2):
    for v in variants:
        os.environ["SPM_HIP_UNIGRAM_VARIANT"] = str(v)
        dm = spm_amd.DeviceModel(mb)
        dm.set_timing(True)
        ms = []
        gen = 0
        for _ in range(6):
            dm.encode_device(d_b.data_ptr(), d_o.data_ptr(), n, d_i.data_ptr(), d_t.data_ptr(),
                             stream=torch.cuda.current_stream(dev).cuda_stream)
            ms.append(dm.stats().fast_kernel_ms)
            gen = dm.stats().general_path
        torch.cuda.synchronize()
        k = int(d_t[-1].item())
        h = (d_i[:k].cpu().numpy().astype(np.int64) * 1000003 % 998244353).sum()
        if ref is None:
            ref = (k, h)
        ok = (k, h) == ref
        print("variant %d: fast kernel %.3f ms (min %.3f) general %d match=%s" % (v, np.mean(ms[1:]), min(ms), gen, ok),
              flush=True)
        dm.close()
