"""The C-ABI libraries load and export every symbol their headers declare (no GPU needed)."""
import ctypes as C
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    with open(os.path.join(REPO, "include", header)) as fh:
        src = fh.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b((?:bc|bcio)_[a-z0-9_]+)\s*\(", src)))


@pytest.mark.parametrize("header,lib", [("basecount_hip.h", "libbasecount_hip.so"),
                                        ("bcio.h", "libbcio.so")])
def test_library_exports_every_declared_symbol(header, lib):
    names = _declared(header)
    assert len(names) >= 10
    L = C.CDLL(os.path.join(REPO, "basecount_amd", lib))
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_hip_library_reports_no_device_without_gpu():
    from basecount_amd import device as D

    assert D.lib().bc_abi_version() == 8
    # the shipped build has no work-skipping diagnostics compiled in
    assert D.build_info().startswith("gfx950") and "diag=0" in D.build_info()
    n = D.device_count()
    if n == 0:
        with pytest.raises(D.BcError) as ei:
            D.Context(0)
        assert ei.value.code == D.BC_E_NODEV


def test_hip_library_contains_gfx950_code_object():
    with open(os.path.join(REPO, "basecount_amd", "libbasecount_hip.so"), "rb") as fh:
        blob = fh.read()
    assert b"gfx950" in blob


def test_hip_library_rejects_null_arguments_without_touching_a_device():
    """Argument checks come first: NULL contexts / outputs are BC_E_ARG with a message."""
    from basecount_amd import device as D

    L = D.lib()
    assert L.bc_ctx_wait(None, None) == D.BC_E_ARG
    assert b"NULL" in L.bc_last_error()
    assert L.bc_sync(None) == D.BC_E_ARG
    assert L.bc_ctx_set_shape(None, 0, 0, 0) == D.BC_E_ARG
    assert L.bc_ctx_release_scratch(None) == D.BC_E_ARG
    assert L.bc_pileup(None, None, 0, 0, 5, 0.0, 0.0, None, None, None, None, None) == D.BC_E_ARG
