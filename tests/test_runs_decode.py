"""The read-chunked kernel's fast CIGAR decode (decode_fast2, basecount_amd/csrc/bc_runs.h) against
the run-table decoder (decode_runs<2>), compiled for the host from the same header: every field
k_rc reads is identical whenever the fast decode accepts a read (count.cpp:40-96 semantics)."""
import os
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fast_decode_matches_run_tables():
    src = os.path.join(REPO, "tests", "native", "runs_check.cpp")
    with tempfile.TemporaryDirectory() as tmp:
        exe = os.path.join(tmp, "runs_check")
        try:
            subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-I",
                            os.path.join(REPO, "basecount_amd", "csrc"), src, "-o", exe],
                           check=True, capture_output=True, text=True)
        except FileNotFoundError:
            pytest.skip("no g++")
        r = subprocess.run([exe, "400000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
