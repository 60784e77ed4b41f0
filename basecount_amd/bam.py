"""Host BAM access: native BGZF/BAM decoder -> numpy struct-of-arrays.

Replaces the pysam calls of the reference read loop (``/root/reference/basecount/main.py:95-127``,
``:165-173``).  ``BamFile`` decodes the whole file once (multi-threaded inflate) and exposes the
records as numpy views; ``select()`` reproduces the read filter of ``main.py:165`` and groups the
accepted reads per reference in the GPU batch layout (``basecount_hip.h: bc_reads``).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _native as N

_NP = {
    np.int32: C.c_int32, np.uint32: C.c_uint32, np.int64: C.c_int64, np.uint64: C.c_uint64,
    np.uint16: C.c_uint16, np.uint8: C.c_uint8,
}


def _view(ptr: int, n: int, dtype) -> np.ndarray:
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    ct = _NP[dtype]
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(int(n),))


REC_NO_CIGAR, REC_NO_SEQ, REC_NO_QUAL, REC_BAD_CLIP, REC_NEG_POS = 1, 2, 4, 8, 16

SEQ_NT16 = "=ACMGRSVTWYHKDBN"


@dataclass
class Selection:
    """Accepted reads of the requested references (flat arrays sliced by ``ref_beg``).  Like the
    record arrays of BamFile, these are views of the decoder's memory (each select() call gets
    its own block): valid until the BamFile is closed."""

    n_accepted: int
    keyerror_ordinal: int
    keyerror_rec: int
    ref_beg: np.ndarray
    pos: np.ndarray
    cig_beg: np.ndarray
    cig_n: np.ndarray
    seq_nib: np.ndarray
    qlen: np.ndarray
    ordinal: np.ndarray
    rec: np.ndarray
    span: np.ndarray  # int64 reference span (M/D/N/=/X) of each selected read


class BamFile:
    """A fully decoded BAM file (records in file order), or one batch of a BamStream (then its
    record indices count from the batch's first record, ``first_record`` in the file)."""

    def __init__(self, path: str | None, nthreads: int = 0, *, _handle=None, _first: int = 0):
        lib = N.bcio()
        if _handle is None:
            h = C.c_void_p()
            rc = lib.bcio_open(os.fsencode(path), int(nthreads), C.byref(h))
            if rc == -1:
                raise FileNotFoundError(lib.bcio_last_error().decode())
            N.bcio_check(rc)
        else:
            h = _handle
        self._h = h
        self.first_record = int(_first)
        nr = lib.bcio_n_refs(h)
        self.references = tuple(lib.bcio_ref_name(h, i).decode() for i in range(nr))
        self.lengths = tuple(int(lib.bcio_ref_len(h, i)) for i in range(nr))
        r = N.BcioRecords()
        N.bcio_check(lib.bcio_get_records(h, C.byref(r)))
        n = r.n
        self.n_records = n
        self.tid = _view(r.tid, n, np.int32)
        self.pos = _view(r.pos, n, np.int32)
        self.flag = _view(r.flag, n, np.uint16)
        self.mapq = _view(r.mapq, n, np.uint8)
        self.l_seq = _view(r.l_seq, n, np.int32)
        self.qstart = _view(r.qstart, n, np.int32)
        self.qend = _view(r.qend, n, np.int32)
        self.rec_err = _view(r.rec_err, n, np.uint32)
        self.cig_off = _view(r.cig_off, n + 1, np.uint64)
        self.cigar = _view(r.cigar, int(self.cig_off[-1]) if n else 0, np.uint32)
        self.seq_off = _view(r.seq_off, n + 1, np.uint64)
        self.seq = _view(r.seq, int(r.seq_bytes), np.uint8)
        self.qual = _view(r.qual, 2 * int(r.seq_bytes), np.uint8)
        self.ref_span = _view(r.ref_span, n, np.int64)
        # SEQ in the kernels' BC_SEQ_EVENT layout, padded (uploaded as is: no device pass)
        self.seq_event = _view(r.seq_event, int(r.seq_event_bytes), np.uint8)

    def close(self) -> None:
        if getattr(self, "_h", None):
            N.bcio().bcio_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def select(self, min_mapping_quality: int, ref_selected) -> Selection:
        """Accepted reads (``not is_unmapped and mapq >= mmq``) grouped by reference."""
        sel = np.ascontiguousarray(np.asarray(ref_selected, dtype=np.uint8))
        if sel.size != len(self.references):
            raise ValueError("ref_selected must have one entry per reference")
        o = N.BcioSelection()
        mmq = max(min(int(min_mapping_quality), 1 << 40), -(1 << 40))
        N.bcio_check(
            N.bcio().bcio_select(self._h, mmq, sel.ctypes.data if sel.size else None, C.byref(o))
        )
        nr = len(self.references)
        ref_beg = _view(o.ref_beg, nr + 1, np.int64).copy()
        m = int(ref_beg[-1])
        return Selection(
            n_accepted=int(o.n_accepted),
            keyerror_ordinal=int(o.keyerror_ordinal),
            keyerror_rec=int(o.keyerror_rec),
            ref_beg=ref_beg,
            pos=_view(o.pos, m, np.int32),
            cig_beg=_view(o.cig_beg, m, np.uint32),
            cig_n=_view(o.cig_n, m, np.uint32),
            seq_nib=_view(o.seq_nib, m, np.uint32),
            qlen=_view(o.qlen, m, np.uint32),
            ordinal=_view(o.ordinal, m, np.int64),
            rec=_view(o.rec, m, np.int64),
            span=_view(o.span, m, np.int64),
        )

    # ---- pysam-like per-record accessors (tests / oracle shim only; slow) -------------------
    def cigartuples(self, i: int):
        a, b = int(self.cig_off[i]), int(self.cig_off[i + 1])
        if a == b:
            return None
        return [(int(w) & 0xF, int(w) >> 4) for w in self.cigar[a:b]]

    def query_alignment_sequence(self, i: int):
        ls = int(self.l_seq[i])
        if ls == 0:
            return None
        qs, qe = int(self.qstart[i]), int(self.qend[i])
        base = 2 * int(self.seq_off[i])
        idx = np.arange(max(qs, 0), max(qe, 0)) if qe > qs else np.zeros(0, dtype=np.int64)
        nib = self._nibbles(base, idx)
        return "".join(SEQ_NT16[v] for v in nib)

    def query_alignment_qualities(self, i: int):
        ls = int(self.l_seq[i])
        if ls == 0:
            return None
        base = 2 * int(self.seq_off[i])
        if self.qual[base] == 0xFF:
            return None
        qs, qe = int(self.qstart[i]), int(self.qend[i])
        if qe <= qs:
            return self.qual[base:base].copy()
        return self.qual[base + qs : base + qe].copy()

    def _nibbles(self, base_nib: int, idx: np.ndarray) -> np.ndarray:
        j = base_nib + idx
        byte = self.seq[j >> 1]
        return np.where(j & 1, byte & 0xF, byte >> 4)


def find_ref_start(path: str, tid: int, pos: int | None = None) -> int | None:
    """Virtual offset of the first record whose refID is >= tid or -1 (with ``pos``: the first
    at or past (tid, pos) in coordinate order), None if the file ends first; found without
    inflating the file (bcio_find_ref_start / bcio_find_record).  Exact for a coordinate-sorted
    file; BamStream(voff_range=...) streams verify a split (a wrong one fails their decode)."""
    lib = N.bcio()
    v = C.c_uint64()
    if pos is None:
        rc = lib.bcio_find_ref_start(os.fsencode(path), int(tid), C.byref(v))
    else:
        rc = lib.bcio_find_record(os.fsencode(path), int(tid), int(pos), C.byref(v))
    if rc == -1:
        raise FileNotFoundError(lib.bcio_last_error().decode())
    N.bcio_check(rc)
    return int(v.value) or None


class BamStream:
    """A BAM file decoded in batches of records (file order) with bounded memory: the
    reference's chunked read loop (main.py:142-162) without holding the file.

        with BamStream(path) as s:
            for batch in s.batches(1_000_000):   # BamFile per batch, closed when the next comes
                ...
    """

    def __init__(self, path: str, nthreads: int = 0, *, voff_range: tuple | None = None):
        """``voff_range=(begin, end)``: only the records in [begin, end) (BAM virtual offsets,
        ``find_ref_start``; end None: to the end of the file, begin None: no records)."""
        lib = N.bcio()
        h = C.c_void_p()
        if voff_range is None:
            rc = lib.bcio_stream_open(os.fsencode(path), int(nthreads), C.byref(h))
        else:
            beg, end = voff_range
            if beg is None:  # an empty range
                beg, end = 1, 1
            rc = lib.bcio_stream_open_range(os.fsencode(path), int(nthreads), int(beg), int(end or 0), C.byref(h))
        if rc == -1:
            raise FileNotFoundError(lib.bcio_last_error().decode())
        N.bcio_check(rc)
        self._h = h
        nr = lib.bcio_stream_n_refs(h)
        self.references = tuple(lib.bcio_stream_ref_name(h, i).decode() for i in range(nr))
        self.lengths = tuple(int(lib.bcio_stream_ref_len(h, i)) for i in range(nr))

    def next_batch(self, max_records: int) -> BamFile | None:
        lib = N.bcio()
        first = int(lib.bcio_stream_records(self._h))
        out = C.c_void_p()
        N.bcio_check(lib.bcio_stream_next(self._h, int(max_records), C.byref(out)))
        if not out.value:
            return None
        return BamFile(None, _handle=out, _first=first)

    def batches(self, max_records: int):
        """Yield the batches; each is closed when the next one is requested."""
        prev = None
        try:
            while True:
                b = self.next_batch(max_records)
                if prev is not None:
                    prev.close()
                prev = b
                if b is None:
                    return
                yield b
        finally:
            if prev is not None:
                prev.close()

    def close(self) -> None:
        if getattr(self, "_h", None):
            N.bcio().bcio_stream_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def write_bam(path, references, lengths, tid, pos, flag, mapq, cig_off, cigar, l_seq, seq_off,
              seq, qual_off, qual, level: int = 1, nthreads: int = 0) -> None:
    """Serialise records (CSR arrays) into a BGZF-compressed BAM file."""
    arrs = dict(
        tid=np.ascontiguousarray(tid, np.int32), pos=np.ascontiguousarray(pos, np.int32),
        flag=np.ascontiguousarray(flag, np.uint16), mapq=np.ascontiguousarray(mapq, np.uint8),
        cig_off=np.ascontiguousarray(cig_off, np.uint64),
        cigar=np.ascontiguousarray(cigar, np.uint32),
        l_seq=np.ascontiguousarray(l_seq, np.int32),
        seq_off=np.ascontiguousarray(seq_off, np.uint64), seq=np.ascontiguousarray(seq, np.uint8),
        qual_off=np.ascontiguousarray(qual_off, np.uint64),
        qual=np.ascontiguousarray(qual, np.uint8),
    )
    n = arrs["tid"].size
    names = (C.c_char_p * max(1, len(references)))(*[r.encode() for r in references])
    lens = np.ascontiguousarray(lengths, np.int64)
    spec = N.BcioWriteSpec()
    spec.n_refs = len(references)
    spec.ref_names = names
    spec.ref_lens = lens.ctypes.data
    spec.n = n
    for k, v in arrs.items():
        setattr(spec, k, v.ctypes.data)
    spec.level = int(level)
    spec.nthreads = int(nthreads)
    N.bcio_check(N.bcio().bcio_write_bam(os.fsencode(path), C.byref(spec)))


def seq_event_bytes(nbytes: int) -> int:
    """Size of the padded BC_SEQ_EVENT buffer for nbytes of BAM-packed SEQ."""
    return (int(nbytes) + 15) // 16 * 16 + 16


def seq_to_event(seq: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """BAM-packed SEQ bytes -> the kernels' BC_SEQ_EVENT layout (padded), on the host."""
    src = np.ascontiguousarray(seq, np.uint8)
    out = np.empty(seq_event_bytes(src.size), np.uint8)
    N.bcio_check(N.bcio().bcio_seq_to_event(src.ctypes.data if src.size else None, src.size,
                                            out.ctypes.data, out.size, int(nthreads)))
    return out


def pack_seq(seq_str: str) -> np.ndarray:
    """ASCII bases -> BAM 4-bit packed bytes (high nibble first)."""
    lut = np.zeros(256, np.uint8)
    for code, ch in enumerate(SEQ_NT16):
        lut[ord(ch)] = code
        lut[ord(ch.lower())] = code
    codes = lut[np.frombuffer(seq_str.encode("ascii"), np.uint8)]
    if codes.size % 2:
        codes = np.concatenate([codes, np.zeros(1, np.uint8)])
    return (codes[0::2] << 4) | codes[1::2]
