"""Host sanitizers: the product's host sources
that read untrusted bytes — model_proto.cc (.model files), double_array.cc
(trie build and walks) and normalizer.cc (the precompiled charsmap blob,
PrefixMatcher) — built with AddressSanitizer + UndefinedBehaviorSanitizer
(tools/sanitize/Makefile, g++ -fsanitize=address,undefined,
-fno-sanitize-recover) and driven over the reference's model files intact,
truncated, bit-flipped, and with corrupted charsmap blobs
(tools/sanitize/driver.cc).  Any report aborts the driver."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_host_sources_asan_ubsan_clean():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools", "sanitize")], timeout=600)
    exe = os.path.join(ROOT, "tools", "bin", "sanitize_driver")
    env = dict(os.environ, SANITIZE_CASES="40,40,200",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    models = [os.path.join(GOLD, m) for m in ("test_model.model", "botchan_bpe1k.model", "test_ja_model.model")]
    p = subprocess.run([exe, os.path.join(GOLD, "botchan.txt")] + models, capture_output=True, timeout=900, env=env)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-4000:]
    res = json.loads(p.stdout.decode().strip().splitlines()[-1])
    assert res["parsed"] > 100 and res["rejected"] > 10 and res["normalized_bytes"] > 0


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("variant", ["trie_check", "trie_check_tsan"])
def test_trie_build_sanitized(variant):
    """double_array.cc's threaded subtree placement: every key and 4000
    random prefix queries per key set against a std::map (ASan+UBSan, TSan)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools", "sanitize")], timeout=600)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    p = subprocess.run([os.path.join(ROOT, "tools", "bin", variant)], capture_output=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-4000:]
    res = json.loads(p.stdout.decode().strip().splitlines()[-1])
    assert res["sets"] == 24 and res["queries"] > 50000
