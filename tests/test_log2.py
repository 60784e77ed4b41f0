"""The kernels' log2 (basecount_amd/csrc/bc_log2.h: glibc's e_log2.c algorithm with the constants
of bc_log2_table.h) built for the host is bit-identical to the C library's log2, i.e. to CPython's
math.log2 that the reference's entropies use (main.py:10-11).  The GPU build of the same header
is checked against the oracle in tests/test_gpu_parity.py (entropies bit-identical)."""
import math
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_build_matches_libm_log2(tmp_path):
    exe = str(tmp_path / "log2_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                    "-I", os.path.join(REPO, "basecount_amd", "csrc"),
                    os.path.join(REPO, "tests", "native", "log2_check.cpp"), "-o", exe, "-lm"],
                   check=True)
    n, bad = map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split())
    assert n > 3_000_000 and bad == 0


def test_libm_log2_is_cpythons():
    """The premise: math.log2 and the C library agree (CPython calls log2 directly)."""
    import ctypes

    libm = ctypes.CDLL("libm.so.6")
    libm.log2.restype = ctypes.c_double
    libm.log2.argtypes = [ctypes.c_double]
    for c, cov in ((1, 3), (2, 3), (7, 9), (123, 4567), (1, 2999999), (5, 5)):
        x = c / cov
        assert libm.log2(x) == math.log2(x)
