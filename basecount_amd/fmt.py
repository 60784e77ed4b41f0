"""Byte-exact text output (main.py:454-499,553-595).

Per-position rows go through the native formatter (``bcio_fmt_rows``), which reproduces
``str(round(x, dp))`` of CPython 3.10 for the ints and floats the reference emits.  Decimal
places outside [0, 323] (where CPython's round() takes other branches) use the pure-Python path.
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import _native as N

BASES = ["A", "C", "G", "T", "DS", "N"]


def rows_text(ref: str, counts: np.ndarray, pc: np.ndarray, ent: np.ndarray, sec: np.ndarray,
              dp: int, long_format: bool, nthreads: int = 0) -> bytes:
    """TSV body for one reference.  counts: int32 [k][L]; pc: f64 [k][L]; ent/sec: f64 [L]."""
    k, L = counts.shape
    if not (0 <= dp <= 323):
        return _rows_text_py(ref, counts, pc, ent, sec, dp, long_format)
    lib = N.bcio()
    h = C.c_void_p()
    N.bcio_check(lib.bcio_fmt_new(C.byref(h)))
    try:
        c = np.ascontiguousarray(counts, np.int32)
        p = np.ascontiguousarray(pc, np.float64)
        e = np.ascontiguousarray(ent, np.float64)
        s = np.ascontiguousarray(sec, np.float64)
        N.bcio_check(lib.bcio_fmt_rows(h, ref.encode(), L, k, c.ctypes.data, p.ctypes.data,
                                       e.ctypes.data, s.ctypes.data, int(dp), int(long_format),
                                       int(nthreads)))
        ptr, size = C.c_void_p(), C.c_int64()
        N.bcio_check(lib.bcio_fmt_take(h, C.byref(ptr), C.byref(size)))
        return C.string_at(ptr.value, size.value) if size.value else b""
    finally:
        lib.bcio_fmt_free(h)


def typed_row_values(counts_col, pc_col, e, s, k):
    """Python-typed values of one position (ints where the reference has ints)."""
    cov = int(sum(counts_col))
    cnt = [int(v) for v in counts_col]
    if cov == 0:
        return cov, cnt, [-1] * k, 1, 1
    nz = sum(1 for v in cnt if v)
    return cov, cnt, [float(v) for v in pc_col], float(e), (1 if nz <= 1 else float(s))


def _rows_text_py(ref, counts, pc, ent, sec, dp, long_format) -> bytes:
    k, L = counts.shape
    out = []
    for p in range(L):
        cov, cnt, pcs, e, s = typed_row_values(counts[:, p], pc[:, p], ent[p], sec[p], k)
        if long_format:
            for j in range(k):
                row = [ref, p + 1, cov, BASES[j], cnt[j], pcs[j], e, s]
                out.append("\t".join(str(round(x, dp)) if not isinstance(x, str) else x
                                     for x in row))
        else:
            row = [ref, p + 1, cov] + cnt + pcs + [e, s]
            out.append("\t".join(str(round(x, dp)) if not isinstance(x, str) else x for x in row))
    return ("\n".join(out) + ("\n" if out else "")).encode()


def write_bytes(data: bytes) -> None:
    """Write to sys.stdout exactly as print() would (binary layer when there is one)."""
    out = sys.stdout
    buf = getattr(out, "buffer", None)
    if buf is not None:
        out.flush()
        buf.write(data)
        buf.flush()
    else:
        out.write(data.decode())


def pyround_native(x: float, dp: int) -> str:
    b = C.create_string_buffer(512)
    n = N.bcio().bcio_fmt_pyround_float(float(x), int(dp), b, 512)
    if n < 0:
        N.bcio_check(n)
    return b.value.decode()
