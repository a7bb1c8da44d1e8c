"""Stamps tying a PMC summary to the kernels it measured.

src_sha256(): sha256 over the device sources of libspm_hip.so (every csrc
*.hip and *.h, the launch-side spm_hip_api.cc and the Makefile, in name
order).  tools/pmc_traffic.py writes it into each summary; bench.py takes a
summary's traffic only when the stamp equals the sources it runs, so a
summary of an older kernel can never be reported as the shipped one's.
lib_sha256(): the built library's hash, recorded beside it (a rebuild of the
same sources may differ in non-code bytes, so it is informational)."""
import glob
import hashlib
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sentencepiece-comments_amd", "csrc")
LIB = os.path.join(ROOT, "sentencepiece-comments_amd", "lib", "libspm_hip.so")


def src_files():
    fs = glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h"))
    fs += [os.path.join(CSRC, "spm_hip_api.cc"), os.path.join(ROOT, "sentencepiece-comments_amd", "Makefile")]
    return sorted(fs, key=os.path.basename)


def src_sha256():
    h = hashlib.sha256()
    for f in src_files():
        h.update(os.path.basename(f).encode() + b"\0")
        h.update(open(f, "rb").read())
    return h.hexdigest()


def lib_sha256():
    if not os.path.exists(LIB):
        return None
    return hashlib.sha256(open(LIB, "rb").read()).hexdigest()


def git_head():
    try:
        out = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], stdout=subprocess.PIPE,
                             stderr=subprocess.DEVNULL, timeout=10)
        return out.stdout.decode().strip() or None
    except Exception:
        return None


def slug(kernel_substr):
    return re.sub(r"[^A-Za-z0-9]+", "_", kernel_substr).strip("_")


def steady_bytes(pmc, drop_last=False):
    """Bytes per launch: the mean over the dispatches, or (E-step PARITY,
    `steady` = "low2of3") the median of the lower two thirds — the first chunk
    of every epoch keeps every record and is not the steady state.
    drop_last (the encode legs): the mean without the last dispatch, which is
    bench.py's blocking call after the timed region (the general-path count
    and the parity check's piece lengths: it also writes a length per token,
    so it is not the timed launch's traffic)."""
    r, w = pmc.get("read_bytes_per_dispatch"), pmc.get("write_bytes_per_dispatch")
    if pmc.get("steady") == "low2of3" and r and w and len(r) == len(w):
        tot = sorted(a + b for a, b in zip(r, w))
        low = tot[: max(1, (2 * len(tot)) // 3)]
        return low[len(low) // 2]
    if drop_last and r and w and len(r) == len(w) and len(r) >= 2:
        tot = [a + b for a, b in zip(r, w)][:-1]
        return sum(tot) / len(tot)
    return pmc["hbm_bytes_per_launch"]
