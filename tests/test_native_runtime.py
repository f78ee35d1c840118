"""Native host-runtime self-test (csrc/tests/runtime_selftest.cpp) built plain and under
AddressSanitizer + UndefinedBehaviorSanitizer.  Covers the C++ JSON parser,
safetensors writer/reader incl. 200 corrupted-header variants, byte-level / SentencePiece BPE
round trips, the token dataset (DP sharding, resume) and the PowerMonitor policy."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_runtime_selftest_asan_ubsan(tmp_path):
    r = subprocess.run(["bash", os.path.join(REPO, "scripts", "sanitize_runtime.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "sanitized runtime selftest OK" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr
