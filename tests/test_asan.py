"""The host sanitizer run (scripts/asan.sh): libbcio and the oracle's C code rebuilt
with AddressSanitizer + UBSan, and the CPU tests that drive them (BAM round trips, hostile
BGZF/BAM inputs, formatter, oracle vs the reference's golden vectors) must pass clean."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc with libasan")
def test_host_code_clean_under_asan_ubsan():
    r = subprocess.run(["bash", os.path.join(REPO, "scripts", "asan.sh")], capture_output=True,
                       text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and "ERROR: AddressSanitizer" not in tail, tail
