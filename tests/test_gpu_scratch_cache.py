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
