"""A/B of the cooperative kernel on the Japanese leg's corpus (wagahaiwa x
427 = 1 M lines, test_ja_model.model): the coop path's HIP-event time per
blocking call for each setting given on the command line, e.g.
  python tools/coop_ab.py slab=1 slab=2 slab=1,blocks=1024
(slab = spm_hip_model_set_coop_slab mode; blocks = SPM_HIP_COOP_BLOCKS, read
per call).  With SPM_HIP_COOP_PROF=1 the library prints phase cycles."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sentencepiece-comments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import oracle_lib  # noqa: E402
if os.environ.get("AB_OLD"):  # another build's library (ablib/<AB_OLD>: libspm_hip_<tag>.so + spm_amd_<tag>.py)
    import importlib
    tag = os.environ["AB_OLD"] if os.environ["AB_OLD"] != "1" else "r05"
    sys.path.insert(0, os.path.join(ROOT, "ablib"))
    os.environ["SPM_AMD_LIB"] = os.path.join(ROOT, "ablib", "libspm_hip_%s.so" % tag)
    spm_amd = importlib.import_module("spm_amd_%s" % tag)
else:
    import spm_amd  # noqa: E402


def main():
    gold = os.path.join(ROOT, "tests", "golden")
    mb = open(os.path.join(gold, "test_ja_model.model"), "rb").read()
    lines = oracle_lib.read_lines_binary(os.path.join(gold, "wagahaiwa_nekodearu.txt"))
    hm = spm_amd.DeviceModel(mb, host_only=True)
    rb, ro = spm_amd.to_csr(lines)
    nb, no = hm.normalize_csr(rb, ro, threads=16)
    hm.close()
    reps = 427
    ln = (no[1:] - no[:-1]).astype(np.uint64)
    lens = np.tile(ln, reps)
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens, dtype=np.uint64)
    buf = np.tile(nb[:int(no[-1])], reps)
    dev = torch.device("cuda", 0)
    d_b = torch.from_numpy(buf).to(dev)
    d_o = torch.from_numpy(off.view(np.int64)).to(dev)
    n = len(lens)
    d_ids = torch.empty(int(off[-1]), dtype=torch.int32, device=dev)
    d_tok = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ref = None
    for arg in sys.argv[1:]:
        kv = dict(x.split("=", 1) for x in arg.split(",") if "=" in x)
        if "blocks" in kv:
            os.environ["SPM_HIP_COOP_BLOCKS"] = kv["blocks"]
        else:
            os.environ.pop("SPM_HIP_COOP_BLOCKS", None)
        dm = spm_amd.DeviceModel(mb)
        dm.set_timing(True)
        if hasattr(dm, "set_coop_slab"):
            dm.set_coop_slab(int(kv.get("slab", 0)))
        ms = []
        for it in range(4):
            dm.encode_device(d_b.data_ptr(), d_o.data_ptr(), n, d_ids.data_ptr(), d_tok.data_ptr())
            st = dm.stats()
            if it:
                ms.append(st.general_kernel_ms)
        torch.cuda.synchronize()
        got = (d_tok.cpu().numpy().copy(), d_ids[:int(d_tok[-1].item())].cpu().numpy().copy())
        if ref is None:
            ref = got
        same = np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])
        lib, _ = spm_amd.device_bytes()
        print("%-24s coop path %.2f ms (min %.2f)  rest %d  same-as-first %s  lib bytes %.3g" %
              (arg, float(np.mean(ms)), float(np.min(ms)), getattr(st, "coop_rest", -1), same, float(lib)),
              flush=True)
        dm.close()


if __name__ == "__main__":
    main()
