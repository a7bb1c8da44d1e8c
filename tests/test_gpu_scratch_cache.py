"""The trainer's device scratch cache (csrc/scratch_cache.{h,cc}): carving
best fit, coalescing, disjoint ranges, event-ordered reuse and release —
ADVICE r03 (a small request must not pin a large cached block; no
device-wide sync per free).  The checks live in the native selftest."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "sentencepiece-comments_amd", "lib", "scratch_cache_selftest")


@pytest.mark.gpu
def test_scratch_cache_selftest():
    assert os.path.exists(EXE), "build with __graft_entry__.build()"
    p = subprocess.run([EXE], capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert p.stdout.decode().strip() == "ok"


@pytest.mark.gpu
def test_device_bytes_accounting():
    """spm_hip_device_bytes: a model's blocks count while it lives and are
    returned when it is freed; the peak covers the encode workspace."""
    import numpy as np
    import spm_amd as S
    import synth
    live0, _ = S.device_bytes()
    S.device_peak_reset()
    dm = S.DeviceModel(open(os.path.join(ROOT, "data", "synth32k_unigram.model"), "rb").read())
    live1, _ = S.device_bytes()
    assert live1 > live0
    buf, off = synth.normalized(20000, seed=3)
    dm.encode_csr_host(buf, off)
    live2, peak = S.device_bytes()
    assert peak >= live2 >= live1 and peak > int(off[-1])
    dm.close()
    assert S.device_bytes()[0] == live0
