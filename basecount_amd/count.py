"""Drop-in for the reference's native module ``count`` (count.cpp:102-105, setup.py:5).

    from basecount_amd.count import bcount      # instead of: from count import bcount

``bcount(refLen, minBaseQuality, reads, qualities, starts, ctuples) -> list[list[int]]`` takes the
same positional arguments (pysam's query_alignment_sequence strings, query_alignment_qualities
arrays, reference_start ints and cigartuples lists) and returns the same refLen x 6 list of
[A, C, G, T, DS, N] counts.  The Python lists are packed into the HBM batch layout (4-bit SEQ,
CIGAR words) and counted by kernel 1 through ``bc_bcount_host``.

Errors follow pybind11 / the C++ (count.cpp:60-65,85): unconvertible arguments (None, negative or
>= 2^32 integers, non-str reads) raise ``TypeError``; a counted base or deletion past the reference
end raises ``IndexError("vector::_M_range_check: ...")``.  Where the reference's behaviour is
undefined (a CIGAR consuming more bases than the read holds, lists of different lengths) this
raises ``ValueError`` instead of reading out of bounds.
"""
from __future__ import annotations

import ctypes as C
from itertools import chain

import numpy as np

from . import device as D
from .main import _SIG, default_device

_U32 = 1 << 32
# ASCII letter -> BAM 4-bit code; only A C G T N are ever counted (count.cpp:58-65), every
# other byte maps to 0 ('='), which counts nowhere.
_LUT = np.zeros(256, np.uint8)
for _ch, _code in (("A", 1), ("C", 2), ("G", 4), ("T", 8), ("N", 15)):
    _LUT[ord(_ch)] = _code


def _type_error(args):
    return TypeError(_SIG + ", ".join(repr(a) for a in args))


def _as_u32(x, args) -> int:
    if isinstance(x, float) or not hasattr(x, "__index__") and not hasattr(x, "__int__"):
        raise _type_error(args)
    try:
        v = int(x)
    except Exception:
        raise _type_error(args) from None
    if not 0 <= v < _U32:
        raise _type_error(args)
    return v


def pack(reads, qualities, starts, ctuples, args=None):
    """Python lists -> host bc_reads dict (4-bit SEQ, nibble-indexed QUAL, CIGAR words)."""
    args = args if args is not None else (None, None, reads, qualities, starts, ctuples)
    n = len(reads)
    if not (len(qualities) >= n and len(starts) >= n and len(ctuples) >= n):
        raise ValueError("reads, qualities, starts and ctuples must have the same length")
    if any(not isinstance(r, str) for r in reads):
        raise _type_error(args)
    if any(q is None for q in qualities[:n]) or any(c is None for c in ctuples[:n]):
        raise _type_error(args)
    lens = np.fromiter((len(r) for r in reads), np.int64, n)
    # each read starts on a byte boundary (like BAM): pad odd reads with one code-0 nibble
    padded = lens + (lens & 1)
    nib_off = np.zeros(n + 1, np.int64)
    np.cumsum(padded, out=nib_off[1:])
    text = "".join(r if len(r) % 2 == 0 else r + "=" for r in reads)
    # one byte per character ('?' for anything outside latin-1, which counts nowhere)
    raw = np.frombuffer(text.encode("latin-1", "replace"), np.uint8)
    codes = _LUT[raw]
    if codes.size % 2:
        codes = np.concatenate([codes, np.zeros(1, np.uint8)])
    seq = ((codes[0::2] << 4) | codes[1::2]).astype(np.uint8)
    qlens = np.fromiter((len(q) for q in qualities[:n]), np.int64, n)
    qual = np.zeros(int(nib_off[-1]), np.uint8)
    if n:
        flat = np.fromiter(chain.from_iterable(qualities[:n]), np.int64, int(qlens.sum()))
        if flat.size and (flat.min() < 0 or flat.max() >= _U32):
            raise _type_error(args)
        dst = np.repeat(nib_off[:-1], qlens) + (np.arange(flat.size) - np.repeat(
            np.concatenate([[0], np.cumsum(qlens)[:-1]]), qlens))
        # qualities above 255 behave like 255 for every threshold < 256 and pass any
        # threshold <= their value; clamp only when no threshold can tell them apart
        qual[dst] = np.minimum(flat, 255).astype(np.uint8)
        qhi = flat.max() > 255 if flat.size else False
    else:
        qhi = False
    cig_n = np.fromiter((len(c) for c in ctuples[:n]), np.int64, n)
    pairs = list(chain.from_iterable(ctuples[:n]))
    if pairs:
        try:
            arr = np.array(pairs, dtype=np.int64).reshape(-1, 2)
        except (TypeError, ValueError):
            raise _type_error(args) from None
        if arr.min() < 0 or arr.max() >= _U32:
            raise _type_error(args)
        if arr[:, 0].max() > 15 or arr[:, 1].max() >= (1 << 28):
            raise ValueError("CIGAR operation or length outside the BAM encoding")
        cigar = ((arr[:, 1] << 4) | arr[:, 0]).astype(np.uint32)
    else:
        cigar = np.zeros(0, np.uint32)
    cig_beg = np.zeros(n, np.int64)
    if n:
        cig_beg[1:] = np.cumsum(cig_n)[:-1]
    st = np.fromiter((_as_u32(s, args) for s in starts[:n]), np.int64, n)
    if st.size and st.max() > 0x7FFFFFFF:
        raise ValueError("start beyond the int32 reference coordinate range")
    # query consumption must fit the read (reference behaviour is undefined beyond it)
    if cigar.size:
        op = cigar & 0xF
        ql = np.where((op == 0) | (op == 1) | (op == 7) | (op == 8), cigar >> 4, 0).astype(np.int64)
        cq = np.zeros(cigar.size + 1, np.int64)
        np.cumsum(ql, out=cq[1:])
        qcons = cq[cig_beg + cig_n] - cq[cig_beg]
        if np.any(qcons > np.minimum(lens, qlens)):
            raise ValueError("a CIGAR consumes more query bases than its read / qualities hold")
    return dict(pos=st.astype(np.int32), cig_beg=cig_beg.astype(np.uint32),
                cig_n=cig_n.astype(np.uint32), seq_nib=nib_off[:-1].astype(np.uint32),
                cigar=cigar, seq=seq, qual=qual, qual_overflow=qhi)


def bcount(refLen, minBaseQuality, reads, qualities, starts, ctuples):
    args = (refLen, minBaseQuality, reads, qualities, starts, ctuples)
    L = _as_u32(refLen, args)
    mbq = _as_u32(minBaseQuality, args)
    b = pack(reads, qualities, starts, ctuples, args)
    if b.pop("qual_overflow") and mbq > 255:
        raise ValueError("qualities above 255 with minBaseQuality above 255 are not supported")
    hr, keep = D.host_reads(b)
    out = np.zeros((max(L, 1), 6), np.uint32)
    bad_read, bad_pos = C.c_int64(-1), C.c_int64(-1)
    rc = D.lib().bc_bcount_host(default_device(), L, mbq, C.byref(hr), out.ctypes.data,
                                C.byref(bad_read), C.byref(bad_pos))
    if rc == D.BC_E_RANGE:
        raise IndexError(D.lib().bc_last_error().decode())
    D.check(rc)
    return out[:L].tolist()
