"""Host orchestration: the reference's Python layer (/root/reference/basecount/main.py) driving the
MI355X kernels.

Same public surface as the reference — ``get_entropy``, ``get_stats``, ``get_references``,
``open_samfile``, ``init_read_chunk``, ``get_basecounts``, ``BaseCount`` (``rows``, ``records``,
``num_reads``, ``mean_coverage``, ``mean_entropy``, ``columns``, ``references``,
``reference_lengths``, ``data``), ``handle_arg`` and the ``run`` CLI — with the same outputs,
argument meanings and exceptions.  What changes is where the work happens:

  reference                                   here
  pysam read loop (main.py:127-174)           native BAM decoder + numpy filter (bam.py)
  count.bcount per chunk (main.py:146,179)    kernel 1 on the whole reference at once (HBM)
  np.add of chunks (main.py:155,188)          device-resident int32 histogram
  get_stats Python loop (main.py:29-78)       kernel 2 (fp64, same operation order)
  summary / amplicon loops (main.py:469-551)  numpy-exact device reductions (bc_summary /
                                              bc_amplicons)

Chunking (``chunk_size``) cannot change counts (integer sums commute); it only decides WHICH
error the reference raises first when the input has several faults, so the same timeline is
replayed from the fault positions (``_first_error``).
"""
from __future__ import annotations

import argparse
import json
import ctypes as C
import math
import os
import sys
from array import array

import numpy as np

from . import device as D
from . import fmt
from .bam import REC_BAD_CLIP, REC_NEG_POS, REC_NO_CIGAR, REC_NO_QUAL, REC_NO_SEQ, BamFile, BamStream, find_ref_start
from .scheme import load_scheme
from .version import __version__

_TYPE_FAULTS = REC_NO_CIGAR | REC_NO_SEQ | REC_NO_QUAL | REC_NEG_POS
_SIG = (
    "bcount(): incompatible function arguments. The following argument types are supported:\n"
    "    1. (arg0: typing.SupportsInt | typing.SupportsIndex, arg1: typing.SupportsInt | "
    "typing.SupportsIndex, arg2: collections.abc.Sequence[str], arg3: collections.abc.Sequence"
    "[collections.abc.Sequence[typing.SupportsInt | typing.SupportsIndex]], arg4: collections."
    "abc.Sequence[typing.SupportsInt | typing.SupportsIndex], arg5: collections.abc.Sequence"
    "[collections.abc.Sequence[tuple[typing.SupportsInt | typing.SupportsIndex, typing."
    "SupportsInt | typing.SupportsIndex]]]) -> list[list[int]]\n\nInvoked with: "
)
_U32 = 1 << 32
_CONTEXTS: dict = {}


def default_device() -> int:
    v = os.environ.get("BASECOUNT_DEVICE")
    if v not in (None, ""):
        return int(v)
    v = os.environ.get("LOCAL_RANK")
    if v not in (None, ""):  # one process per GPU; ranks beyond the GPU count share devices
        return int(v) % max(1, D.device_count())
    return 0


def context(device: int | None = None) -> D.Context:
    dev = default_device() if device is None else int(device)
    ctx = _CONTEXTS.get(dev)
    if ctx is None:
        ctx = _CONTEXTS[dev] = D.Context(dev)
    return ctx


def norm_factors(k: int):
    """main.py:24-25: 1/log2(k), 1/log2(k-1) evaluated exactly as the reference does."""
    return 1 / math.log2(k), 1 / math.log2(k - 1)


# ------------------------------------------------------------------------- API parity helpers
def get_entropy(probabilities):
    """main.py:10-11."""
    return sum([-(x * math.log2(x)) if x != 0 else 0 for x in probabilities])


class RefData:
    """Per-position results of one reference, host-resident (downloaded from HBM).

    counts: int32 [k][L]; pc: f64 [k][L]; ent, sec: f64 [L]; cov: int32 [L]."""

    __slots__ = ("counts", "pc", "ent", "sec", "cov")

    def __init__(self, counts, pc, ent, sec, cov):
        self.counts, self.pc, self.ent, self.sec, self.cov = counts, pc, ent, sec, cov

    @property
    def L(self) -> int:
        return int(self.cov.size)


class Rows:
    """Sequence of the reference's row lists (main.py:57-78), built lazily from a RefData with
    the reference's Python types (ints where it has ints)."""

    def __init__(self, ref: str, d: RefData, long_format: bool):
        self.ref, self.d, self.long = ref, d, long_format
        self.k = d.counts.shape[0]

    def __len__(self):
        return self.d.L * (self.k if self.long else 1)

    def _position(self, p, cnt, pcs, e, s):
        cov = sum(cnt)
        if cov == 0:
            return cov, cnt, [-1] * self.k, 1, 1
        nz = sum(1 for v in cnt if v)
        return cov, cnt, pcs, e, (1 if nz <= 1 else s)

    def __iter__(self):
        d, k, ref = self.d, self.k, self.ref
        cols = [c.tolist() for c in d.counts]
        pcs = [c.tolist() for c in d.pc]
        ent, sec = d.ent.tolist(), d.sec.tolist()
        bases = fmt.BASES[:k]
        for p in range(d.L):
            cov, cnt, pc, e, s = self._position(p, [c[p] for c in cols], [c[p] for c in pcs],
                                                ent[p], sec[p])
            if self.long:
                for j in range(k):
                    yield [ref, p + 1, cov, bases[j], cnt[j], pc[j], e, s]
            else:
                yield [ref, p + 1, cov] + cnt + pc + [e, s]

    def __getitem__(self, i):
        n = len(self)
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(n))]
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("list index out of range")
        p, j = (divmod(i, self.k) if self.long else (i, None))
        d = self.d
        cov, cnt, pc, e, s = self._position(
            p, [int(v) for v in d.counts[:, p]], [float(v) for v in d.pc[:, p]], float(d.ent[p]),
            float(d.sec[p]))
        if self.long:
            return [self.ref, p + 1, cov, fmt.BASES[j], cnt[j], pc[j], e, s]
        return [self.ref, p + 1, cov] + cnt + pc + [e, s]

    def __eq__(self, other):
        return list(self) == list(other)


def get_stats(base_counts, ref, show_n_bases=False, long_format=False):
    """main.py:14-79 on the device (kernel 2).  ``base_counts``: refLen x 6 counts."""
    a = np.asarray(base_counts, dtype=np.int64).reshape(-1, 6)
    if not show_n_bases and isinstance(base_counts, list):
        for bc in base_counts:  # the reference pops N from the caller's lists (main.py:31)
            if isinstance(bc, list):
                bc.pop(5)
    k = 6 if show_n_bases else 5
    d = stats_on_device(np.ascontiguousarray(a[:, :k].T.astype(np.int32)), k)
    return list(Rows(ref, d, long_format))


def stats_on_device(planes: np.ndarray, k: int, device: int | None = None) -> RefData:
    """Kernel 2 over host count planes int32 [k][L] (used by get_stats / the bcount adapter)."""
    ctx = context(device)
    L = planes.shape[1]
    if L == 0:
        return RefData(planes, np.zeros((k, 0)), np.zeros(0), np.zeros(0), np.zeros(0, np.int32))
    hist = ctx.alloc(planes.nbytes).upload(planes)
    outs = _alloc_outputs(ctx, k, L, want_pc=True)
    nf, nf2 = norm_factors(k)
    ctx.stats(hist.ptr, L, k, nf, nf2, outs["cov"].ptr, outs["pc"].ptr, outs["ent"].ptr,
              outs["sec"].ptr)
    return _download(outs, planes.copy(), k, L)


def _alloc_outputs(ctx, k, L, want_pc):
    o = {"cov": ctx.alloc(4 * L), "ent": ctx.alloc(8 * L), "sec": ctx.alloc(8 * L)}
    o["pc"] = ctx.alloc(8 * k * L) if want_pc else None
    return o


class _Scratch:
    """Device buffers reused from reference to reference within one get_basecounts call, grown
    (never shrunk) on demand: at GRCh38 sizes the per-reference outputs are GB-sized, and a
    hipMalloc / hipFree (which synchronises) per reference and buffer cost more than the
    kernels.  Every use is stream-ordered after the previous reference's kernels, and rows are
    downloaded before the next reference starts."""

    def __init__(self, ctx):
        self.ctx, self.bufs = ctx, {}
        self.pending_sort = None  # (unsorted reads, sort memory) whose device flags are unread

    def check_sort(self):
        """The flags of the last device sort (bc_reads_sort_check), read once the reference's
        kernels are done (the stream is synced by then): the sort itself never waits."""
        if self.pending_sort is not None:
            r, mem = self.pending_sort
            self.pending_sort = None
            self.ctx.sort_check(r, mem)

    def get(self, role: str, nbytes: int):
        b = self.bufs.get(role)
        if b is None or b.nbytes < nbytes:
            if b is not None:
                b.free()
            b = self.bufs[role] = self.ctx.alloc(max(16, int(nbytes)))
        return b

    def outputs(self, k, L, want_pc):
        return {"cov": self.get("cov", 4 * L), "ent": self.get("ent", 8 * L), "sec": self.get("sec", 8 * L),
                "pc": self.get("pc", 8 * k * L) if want_pc else None}

    def release(self):
        for b in self.bufs.values():
            b.free()
        self.bufs.clear()


# host phases of get_basecounts (seconds), accumulated; printed by BASECOUNT_HIP_TIMING=1
PHASES: dict = {}


class _phase:
    __slots__ = ("name", "t0")

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        import time

        self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        import time

        PHASES[self.name] = PHASES.get(self.name, 0.0) + time.perf_counter() - self.t0


_SCRATCHES: dict = {}


def _scratch(ctx) -> _Scratch:
    """The device's grow-only scratch, kept from call to call (a hipFree synchronises and costs
    ~2 ms each: releasing a call's dozen buffers cost more than its kernels); give the HBM back
    with release_device_memory()."""
    sc = _SCRATCHES.get(ctx.device)
    if sc is None or sc.ctx is not ctx:
        sc = _SCRATCHES[ctx.device] = _Scratch(ctx)
    return sc


# devices whose scratch a call with _keep_scratch=True asked to keep: a later call without the
# flag leaves it in place, release_device_memory() frees it
_KEPT: set = set()


def release_device_memory(only_unkept: bool = False) -> None:
    """Free the HBM kept for reuse by the CLI and by library calls made with _keep_scratch
    (batch buffers, outputs, and the contexts' own kernel scratch: bc_ctx_release_scratch);
    get_basecounts / BaseCount release what they used when they return (only_unkept: scratch
    some earlier call asked to keep stays)."""
    for dev in list(_SCRATCHES):
        if only_unkept and dev in _KEPT:
            continue
        _SCRATCHES.pop(dev).release()
    for dev, ctx in _CONTEXTS.items():
        if not (only_unkept and dev in _KEPT):
            ctx.release_scratch()
    if not only_unkept:
        _KEPT.clear()


def _download(outs, counts, k, L) -> RefData:
    cov = outs["cov"].download(np.int32, L)
    ent = outs["ent"].download(np.float64, L)
    sec = outs["sec"].download(np.float64, L)
    pc = outs["pc"].download(np.float64, k * L).reshape(k, L)
    return RefData(counts, pc, ent, sec, cov)


def get_references(samfile, references=None):
    """main.py:82-92 (returns a set: its iteration order is the output order)."""
    if references is None:
        references = samfile.references
    else:
        for reference in references:
            if not (reference in samfile.references):
                raise Exception(f"{reference} is not a valid reference")
    return set(references)


def open_samfile(bam):
    """main.py:95-100 (no htslib messages to silence: the decoder is ours)."""
    return BamFile(bam)


def init_read_chunk(references):
    """main.py:103-107 (kept for API parity; the device path does not chunk)."""
    return {ref: {"reads": [], "qualities": [], "starts": [], "ctuples": []} for ref in references}


# ------------------------------------------------------------------------- error timeline
def _pysam_args(f: BamFile, recs):
    reads, quals, starts, ctuples = [], [], [], []
    for r in recs:
        r = int(r)
        reads.append(f.query_alignment_sequence(r))
        q = f.query_alignment_qualities(r)
        quals.append(None if q is None else array("B", q.tobytes()))
        starts.append(int(f.pos[r]))
        ctuples.append(f.cigartuples(r))
    return reads, quals, starts, ctuples


def _bad_pos(f: BamFile, rec: int, mbq: int, L: int) -> int:
    """refPos that the reference's .at() rejects first for record ``rec`` (count.cpp:40-96)."""
    rp = int(f.pos[rec])
    qp = 2 * int(f.seq_off[rec]) + int(f.qstart[rec])
    a, b = int(f.cig_off[rec]), int(f.cig_off[rec + 1])
    for w in f.cigar[a:b].tolist():
        op, ln = w & 15, w >> 4
        if op in (0, 7, 8):
            for _ in range(ln):
                if int(f.qual[qp]) >= mbq:
                    byte = int(f.seq[qp >> 1])
                    nib = byte & 15 if qp & 1 else byte >> 4
                    if nib in (1, 2, 4, 8, 15) and rp >= L:
                        return rp
                rp += 1
                qp += 1
        elif op == 1:
            qp += ln
        elif op in (2, 3):
            for _ in range(ln):
                if rp >= L:
                    return rp
                rp += 1
    return -1


class _Faults:
    """What the reference's read loop (main.py:141-189) would raise, gathered while the file
    streams by: every position is a global accepted-read ordinal (file order), so the batches
    the file is decoded in (bounded memory) need not match the reference's chunks.

      keyerror : (ordinal, reference name) of the first accepted read of an unrequested
                 reference (main.py:166 indexes read_chunk by it)
      clip     : ordinal of the first selected read whose clipping pysam rejects (main.py:167)
      type_ord : ref -> ordinal of its first read with a None field / negative start
      range_   : ref -> (ordinal, refPos) of its first read with a counted event >= ref_len
    """

    def __init__(self):
        self.keyerror = None
        self.clip = None
        self.type_ord = {}
        self.range_ = {}
        self.n_records = 0

    def inloop(self):
        """The first in-loop fault (ordinal, exception) or None (KeyError before ValueError on
        the same read: the chunk is indexed before the sequence is fetched)."""
        out = None
        if self.keyerror is not None:
            out = (self.keyerror[0], KeyError(self.keyerror[1]))
        if self.clip is not None and (out is None or self.clip < out[0]):
            out = (self.clip, ValueError("Invalid clipping in CIGAR string"))
        return out


def _first_error(fl: _Faults, ref_order, lengths, mbq, cs, type_args):
    """Replay the reference's read loop / chunk-flush timeline (main.py:141-189) and return the
    exception it raises first, or None.  ``type_args(ref, lo, hi)``: the pysam-shaped arguments
    of the ref's accepted reads with ordinals in [lo, hi) (hi None: to the end of the file)."""
    mbq_bad = not (0 <= mbq < _U32)
    inloop = fl.inloop()

    def chunk_of(o):
        return o // cs if cs > 0 else 0

    faults = {}  # ref -> (chunk, kind)
    for ref in ref_order:
        cand = []
        if mbq_bad:
            cand.append((0, 0, "type"))
        if fl.type_ord.get(ref, -1) >= 0:
            cand.append((chunk_of(fl.type_ord[ref]), 0, "type"))
        if ref in fl.range_:
            cand.append((chunk_of(fl.range_[ref][0]), 1, "range"))
        if cand:
            faults[ref] = min(cand, key=lambda c: (c[0], c[1]))
    empty_first_flush = cs == 0 and mbq_bad and fl.n_records > 0 and bool(ref_order)
    if empty_first_flush:
        inloop = None  # the empty flush at the first record raises before anything else
    if not faults:
        return inloop[1] if inloop else None
    kf = min(v[0] for v in faults.values())
    if inloop is not None:
        if cs <= 0 or kf >= inloop[0] // cs:
            return inloop[1]
    for ref in ref_order:
        v = faults.get(ref)
        if v is None or v[0] != kf:
            continue
        if v[2] == "type":
            if empty_first_flush:  # bcount(L, mbq, [], [], [], []) at the first record
                reads = ([], [], [], [])
            elif cs > 0:
                reads = type_args(ref, kf * cs, (kf + 1) * cs)
            else:
                reads = type_args(ref, 0, None)
            args = [lengths[ref], mbq] + list(reads)
            return TypeError(_SIG + ", ".join(repr(a) for a in args))
        L = lengths[ref]
        return IndexError(f"vector::_M_range_check: __n (which is {fl.range_[ref][1]}) "
                          f">= this->size() (which is {L})")
    return None


def _type_args(bam, batch_records_, mmq, wanted, ref_index):
    """type_args for _first_error: a second pass over the file (error path only) collecting the
    pysam-shaped arguments of one reference's reads in an ordinal range."""

    def collect(ref, lo, hi):
        t = ref_index[ref]
        out = ([], [], [], [])
        base = 0
        with BamStream(bam) as st:
            for f in st.batches(batch_records_):
                sel = f.select(mmq, wanted)
                b0, b1 = int(sel.ref_beg[t]), int(sel.ref_beg[t + 1])
                ords = sel.ordinal[b0:b1] + base
                m = (ords >= lo) & ((ords < hi) if hi is not None else True)
                for dst, src in zip(out, _pysam_args(f, sel.rec[b0:b1][m])):
                    dst.extend(src)
                base += sel.n_accepted
                if hi is not None and base >= hi:
                    break
        return out

    return collect


# ------------------------------------------------------------------------- device pipeline
class _BatchOnDevice:
    """One decoded batch in HBM: CIGAR words, packed SEQ (BC_SEQ_EVENT), nibble-indexed QUAL and
    the per-read arrays of its selected reads (sliced per reference).  The buffers come from the
    call's grow-only scratch, so batch after batch reuses the same HBM (stream-ordered: a batch's
    upload follows the previous batch's kernels on the one stream)."""

    def __init__(self, ctx: D.Context, f: BamFile, sel, need_qual: bool, scratch):
        self.ctx = ctx
        rec_err = f.rec_err[sel.rec] if sel.rec.size else np.zeros(0, np.uint32)
        faulty = (rec_err & (_TYPE_FAULTS | REC_BAD_CLIP)) != 0
        # faulty reads raise before their counts could matter: give them no CIGAR so the range
        # check only ever reports well-formed reads
        self.cig_n = np.where(faulty, 0, sel.cig_n).astype(np.uint32)
        self.pos = np.where(faulty, 0, sel.pos).astype(np.int32)
        self.sel = sel
        # reference spans per read (for the LDS window bound), from the decoder
        self.span = np.where(faulty, 0, sel.span)
        self.d_cigar = scratch.get("b_cigar", max(4, f.cigar.nbytes)).upload(f.cigar)
        # packed SEQ in the kernels' layout (BC_SEQ_EVENT, padded): the decoder built it while
        # filling the records, so the upload is a plain copy (no device conversion pass)
        assert f.seq_event.size == D.seq_event_bytes(f.seq.nbytes)
        self.d_seq = scratch.get("b_seq", f.seq_event.size).upload(f.seq_event)
        self.d_qual = scratch.get("b_qual", max(4, f.qual.nbytes)).upload(f.qual) if need_qual else None
        self.n_cig, self.n_seq, self.n_qual = f.cigar.size, f.seq.size, f.qual.size
        m = sel.pos.size
        self.d_pos = scratch.get("b_pos", max(4, 4 * m)).upload(self.pos)
        self.d_cb = scratch.get("b_cb", max(4, 4 * m)).upload(sel.cig_beg)
        self.d_cn = scratch.get("b_cn", max(4, 4 * m)).upload(self.cig_n)
        self.d_sn = scratch.get("b_sn", max(4, 4 * m)).upload(sel.seq_nib)

    def reads(self, t: int) -> D.BcReads:
        b0, b1 = int(self.sel.ref_beg[t]), int(self.sel.ref_beg[t + 1])
        r = D.BcReads()
        r.n_reads = b1 - b0
        r.pos = self.d_pos.ptr + 4 * b0
        r.cig_beg = self.d_cb.ptr + 4 * b0
        r.cig_n = self.d_cn.ptr + 4 * b0
        r.seq_nib = self.d_sn.ptr + 4 * b0
        r.cigar = self.d_cigar.ptr
        r.n_cigar_words = self.n_cig
        r.seq = self.d_seq.ptr
        r.seq_bytes = self.n_seq
        r.seq_layout = D.BC_SEQ_EVENT
        if self.d_qual is not None:
            r.qual = self.d_qual.ptr
            r.qual_bytes = self.n_qual
        pos = self.pos[b0:b1]
        r.sorted = int(bool(np.all(pos[1:] >= pos[:-1]))) if b1 - b0 > 1 else 1
        r.max_span = int(min(self.span[b0:b1].max(), 2**31 - 1)) if b1 > b0 else 0
        r.max_end = int((pos.astype(np.int64) + self.span[b0:b1]).max()) if b1 > b0 else 0
        return r


def batch_records(chunk_size: int) -> int:
    """Records per decoded batch: the reference's chunk size (main.py:142, accepted reads held
    in memory at once) bounded to [2^16, 2^24] records, 2^22 when it does not bound anything
    (chunk_size <= 0).  BASECOUNT_BATCH_RECORDS overrides (tests: many tiny batches)."""
    v = os.environ.get("BASECOUNT_BATCH_RECORDS")
    if v:
        return max(1, int(v))
    cs = int(chunk_size)
    return min(max(cs, 1 << 16), 1 << 24) if cs > 0 else 1 << 22


# Host buffers released at the end of the CLI run instead of when the stream ends: giving back a
# GB of decoded batch and inflate buffers (munmap, TLB shootdowns on every core the process runs
# on) right before the formatter stalled its threads by ~65 ms at C3.  None: release at once.
_DEFERRED: list | None = None


def _release(h) -> None:
    if _DEFERRED is not None:
        _DEFERRED.append(h)
    else:
        h.close()


class _Ungrouped(Exception):
    """A reference's reads came back after the reference was finished (the file is not grouped
    by reference): start again, accumulating every reference until the end of the file."""


_UNGROUPED = object()  # _get_basecounts' answer on every rank when some rank hit _Ungrouped


class _ShardMiss(Exception):
    """Sharded decode: this rank's byte range of the file did not hold exactly its references'
    records (file not grouped by reference, or a split the record chain does not confirm)."""


def _shard_decode_on(group) -> bool:
    """BASECOUNT_SHARD_DECODE: 0 every rank decodes the whole file; 1 (default) each rank its
    byte range, falling back to the whole file if a range misses; require: a miss is an error."""
    return group is not None and group.world > 1 and os.environ.get("BASECOUNT_SHARD_DECODE", "1") != "0"


def get_basecounts(bam, references=None, min_base_quality=0, min_mapping_quality=0,
                   chunk_size=1000000, show_n_bases=False, long_format=False, *, device=None,
                   _mode="rows", _tiles=None, _group=None, _keep_scratch=False):
    """main.py:110-205 on the device.  Returns {ref: {"rows": Rows, "num_reads": n}} in the
    reference's (set) order.  ``_mode="summary"`` keeps per-position data in HBM and returns
    the numpy-exact summary (and amplicon) reductions instead of rows.

    The BAM streams through in batches of records (``batch_records(chunk_size)``, the
    reference's chunked read loop): host and HBM memory hold one batch (two while the next is
    decoded) plus the per-reference outputs, not the file.  A reference whose reads all lie in
    one batch takes the fused pileup (kernels 1 + 2 in one pass); one spread over several
    batches is accumulated batch by batch (bc_count) and finished by kernel 2 after its last.

    With ``_group`` (a dist.Group, one process per GPU) the references are sharded over the
    ranks (dist.shard): this rank computes and returns only the ones it owns, and the function
    returns ``(results, owner, order)``; every rank raises the same first error.

    Device memory: the call's HBM scratch (batch buffers, outputs; the results are on the host)
    is released when it returns, unless it runs inside the CLI (run(), one process per command)
    or ``_keep_scratch`` asks to keep it for the next call (release_device_memory() frees it)."""
    try:
        return _get_basecounts_top(bam, references, min_base_quality, min_mapping_quality, chunk_size,
                                   show_n_bases, long_format, device, _mode, _tiles, _group)
    finally:
        if _keep_scratch:
            _KEPT.update(_SCRATCHES)
        elif _DEFERRED is None:
            release_device_memory(only_unkept=True)


def _get_basecounts_top(bam, references, min_base_quality, min_mapping_quality, chunk_size, show_n_bases,
                        long_format, device, _mode, _tiles, _group):
    args = (bam, references, min_base_quality, min_mapping_quality, chunk_size, show_n_bases,
            long_format, device, _mode, _tiles, _group)
    if _shard_decode_on(_group):
        # each rank inflates and decodes only the byte range of its own references (a file
        # grouped by reference); None: some rank's range did not confirm, all decode everything
        res = _get_basecounts(*args, grouped=True, sharded=True)
        if res is not None:
            return res
        if os.environ.get("BASECOUNT_SHARD_DECODE") == "require":  # tests: the split must hold
            raise RuntimeError("sharded decode: a rank's byte range did not hold exactly its references")
        if os.environ.get("BASECOUNT_HIP_TIMING"):
            print(f"basecount[{_group.rank}] sharded decode missed: every rank decodes the file",
                  file=sys.stderr)
    try:
        res = _get_basecounts(*args, grouped=True)
    except _Ungrouped:  # (one process: raised where the reference came back)
        res = _UNGROUPED
    if res is _UNGROUPED:  # with a group, every rank returns it (the ranks vote after the loop)
        return _get_basecounts(*args, grouped=False)
    return res


def _get_basecounts(bam, references, min_base_quality, min_mapping_quality, chunk_size, show_n_bases,
                    long_format, device, _mode, _tiles, _group, grouped, sharded=False):
    stream = BamStream(bam)
    try:
        references = get_references(stream, references)
        names = stream.references
        ref_index = {n: i for i, n in enumerate(names)}
        reference_lengths = {ref: stream.lengths[names.index(ref)] for ref in references}
        ref_order = list(references)
        if _group is not None:
            from .dist import agree_order

            # main.py:92's set order is per process (hash seed): every rank follows rank 0's
            ref_order = agree_order(_group, ref_order)
        mmq = min_mapping_quality
        wanted = [n in references for n in names]
        mbq = int(min_base_quality)
        mbq_ok = 0 <= mbq < _U32
        k = 6 if show_n_bases else 5
        ncols = k  # N is only ever reported with show_n_bases
        owner = None
        mine = ref_order
        t_lo, t_hi = 0, len(names)  # the refIDs this rank's byte range holds (sharded decode)
        split = set()  # references whose reads several ranks count (their histograms are summed)
        open_miss = False  # sharded: this rank's range could not be opened
        ungrouped = False  # with a group: a reference came back after it was finished (this rank)
        if sharded:
            from .dist import BOUND, plan_ranges

            # contiguous coordinate ranges per rank (file order): whole references balanced on
            # the requested lengths, or, when every requested reference is small (C2-C4-like),
            # equal cuts of their positions, one reference's reads split over several ranks.
            # Each rank streams only the bytes of its range (the last: to the end of the file,
            # unmapped reads included)
            cuts, owner_t, split_t = plan_ranges([int(x) for x in stream.lengths], wanted, _group.world,
                                                 int(os.environ.get("BASECOUNT_SPLIT_MAX", str(1 << 22))))
            owner = {r: owner_t[ref_index[r]] for r in ref_order}
            split = {names[t] for t in split_t} & set(ref_order)
            mine = [r for r in ref_order if owner[r] == _group.rank]
            rk = _group.rank
            last = rk == _group.world - 1
            t_lo = cuts[rk][0]
            t_hi = len(names) if last else cuts[rk + 1][0] + (1 if cuts[rk + 1][1] != BOUND else 0)

            def where(c):
                return find_ref_start(bam, c[0]) if c[1] == BOUND else find_ref_start(bam, c[0], c[1])

            with _phase("decode"):
                stream.close()
                try:
                    beg = where(cuts[rk])
                    end = None if last else where(cuts[rk + 1])
                    if beg is None or (end is not None and end <= beg):
                        beg = end = None  # no records in this rank's range
                    stream = BamStream(bam, voff_range=(beg, end))
                except (ValueError, OSError):
                    # a probe or the range open failed on this rank (a damaged block near a cut):
                    # a miss like any other, so every rank falls back to the whole-file decode,
                    # which raises the one process's error on every rank
                    stream = BamStream(bam, voff_range=(None, None))
                    open_miss = True
        elif _group is not None:
            from .dist import shard

            # cost estimate before any read is seen: the per-position outputs (linear in length)
            owner = shard(ref_order, {r: int(reference_lengths[r]) for r in ref_order}, _group.world)
            mine = [r for r in ref_order if owner[r] == _group.rank]
        mine_t = {ref_index[r] for r in mine} | {ref_index[r] for r in split}  # the references counted here
        B = batch_records(chunk_size)
        fl = _Faults()
        nreads = {ref: 0 for ref in ref_order}
        results = {}
        acc = {}  # ref -> device histogram accumulating its batches (int32 [ncols][L])
        finished = set()
        ctx = context(device) if (mbq_ok and (mine or split)) else None
        scratch = _scratch(ctx) if ctx is not None else None
        nf, nf2 = norm_factors(k)

        def tiles_of(ref):
            return _tiles(ref) if _tiles else None

        base = 0  # accepted reads before the current batch (global ordinals; sharded: in the range)
        cur = nxt = None
        miss = False
        split_acc = {}  # split reference -> this rank's histogram of its reads

        def next_batch():
            if not sharded:
                return stream.next_batch(B)
            try:
                return stream.next_batch(B)
            except (ValueError, OSError) as e:  # the record chain did not fit the range
                raise _ShardMiss() from e

        try:
            if open_miss:
                raise _ShardMiss()
            with _phase("decode"):
                cur = next_batch()
            sel_next = None
            while cur is not None:
                f = cur
                if sharded and f.n_records:
                    tids = f.tid
                    if bool(np.any(((tids < t_lo) | (tids >= t_hi)) & (tids != -1))):
                        raise _ShardMiss()
                with _phase("select"):
                    sel = sel_next if sel_next is not None else f.select(mmq, wanted)
                sel_next = None
                fl.n_records += f.n_records
                # in-loop faults (global ordinals); type faults per reference
                if fl.keyerror is None and sel.keyerror_ordinal >= 0:
                    t = int(f.tid[sel.keyerror_rec])
                    fl.keyerror = (base + sel.keyerror_ordinal, names[t] if 0 <= t < len(names) else None)
                rec_err = f.rec_err[sel.rec] if sel.rec.size else np.zeros(0, np.uint32)
                clip = (rec_err & REC_BAD_CLIP) != 0
                if fl.clip is None and clip.any():
                    fl.clip = base + int(sel.ordinal[np.argmax(clip)])
                here = []
                for ref in ref_order:
                    t = ref_index[ref]
                    b0, b1 = int(sel.ref_beg[t]), int(sel.ref_beg[t + 1])
                    if b1 == b0:
                        continue
                    nreads[ref] += b1 - b0
                    m = (rec_err[b0:b1] & _TYPE_FAULTS) != 0
                    if fl.type_ord.get(ref, -1) < 0 and m.any():
                        fl.type_ord[ref] = base + int(sel.ordinal[b0 + int(np.argmax(m))])
                    if t in mine_t:
                        here.append(ref)
                # one batch of look-ahead: a reference absent from the next batch is complete
                # (in a file grouped by reference); none after the reference's first in-loop fault
                with _phase("decode"):
                    nxt = next_batch() if fl.inloop() is None else None
                if ctx is not None and here:
                    if any(r in finished for r in here):
                        raise _ShardMiss() if sharded else _Ungrouped()
                    with _phase("select"):
                        nsel = sel_next = nxt.select(mmq, wanted) if (nxt is not None and grouped) else None
                    with _phase("upload"):
                        bod = _BatchOnDevice(ctx, f, sel, need_qual=mbq > 0, scratch=scratch)
                    t_refs = _phase("kernels + download")
                    t_refs.__enter__()
                    for ref in here:
                        t = ref_index[ref]
                        L = int(reference_lengths[ref])
                        # (a reference split over ranks is never complete on one: accumulated)
                        closed = grouped and ref not in split and (
                            nxt is None or int(nsel.ref_beg[t + 1]) == int(nsel.ref_beg[t]))
                        reads = _indexed(ctx, bod.reads(t), L, scratch)
                        b0 = int(sel.ref_beg[t])
                        if closed and ref not in acc:  # the whole reference in this batch: fused
                            results[ref], bad = _device_reference(
                                ctx, reads, L, mbq, ncols, k, nf, nf2, _mode, tiles_of(ref),
                                _tiles is not None, scratch)
                            finished.add(ref)
                        else:  # kernel 1 into the reference's accumulator
                            if ref not in acc:
                                acc[ref] = ctx.alloc(max(16, 4 * ncols * L))
                                acc[ref].zero()
                            ctx.count(reads, L, mbq, ncols, acc[ref].ptr)
                            bad = ctx.range_error()
                            if closed:
                                results[ref] = _finish_reference(ctx, acc.pop(ref), L, ncols, k, nf, nf2, _mode,
                                                                 tiles_of(ref), _tiles is not None, scratch)
                                finished.add(ref)
                        scratch.check_sort()
                        if bad >= 0 and ref not in fl.range_:
                            fl.range_[ref] = (base + int(sel.ordinal[b0 + bad]),
                                              _bad_pos(f, int(sel.rec[b0 + bad]), mbq, L))
                    t_refs.__exit__()
                    with _phase("device (sync)"):
                        ctx.sync()  # the batch's host arrays may go once its copies are done
                base += sel.n_accepted
                if nxt is None:
                    _release(cur)  # the last batch: released after the output (CLI)
                else:
                    cur.close()
                cur, nxt = nxt, None
            for ref in split:  # summed over the ranks once every rank is done (below)
                if ref in acc:
                    split_acc[ref] = acc.pop(ref)
            if ctx is not None and fl.inloop() is None:
                for ref in mine:
                    if ref in results or ref in split:
                        continue
                    L = int(reference_lengths[ref])
                    if ref in acc:
                        results[ref] = _finish_reference(ctx, acc.pop(ref), L, ncols, k, nf, nf2, _mode,
                                                         tiles_of(ref), _tiles is not None, scratch)
                    else:  # no reads at all
                        results[ref], _ = _device_reference(ctx, _no_reads(), L, mbq, ncols, k, nf, nf2,
                                                            _mode, tiles_of(ref), _tiles is not None, scratch)
        except _ShardMiss:
            miss = True
        except _Ungrouped:
            if _group is None or _group.world == 1:
                raise
            ungrouped = True  # told to the other ranks below, before any other collective
        finally:
            for b in (cur, nxt):
                if b is not None:
                    b.close()
            if ctx is not None:
                ctx.sync()
            for b in acc.values():
                b.free()
        if sharded:
            if not _merge_shards(_group, fl, miss, base, ref_order, names, nreads):
                for b in split_acc.values():
                    b.free()
                return None  # some rank's range did not confirm: every rank decodes the file
        elif _group is not None:
            # a file not grouped by reference may show it on some ranks only: all restart together
            if any(v[0] for v in _group.all_gather_ints([int(ungrouped)])):
                return _UNGROUPED
        if not sharded and _group is not None and mbq_ok:
            # every rank needs every reference's first out-of-range read to raise the same error
            flat = [v for r in ref_order for v in fl.range_.get(r, (-2, -1))]
            alls = _group.all_gather_ints(flat)
            fl.range_ = {}
            for i, r in enumerate(ref_order):
                o, bp = alls[owner[r]][2 * i], alls[owner[r]][2 * i + 1]
                if o >= 0:
                    fl.range_[r] = (o, bp)
        try:
            err = _first_error(fl, ref_order, reference_lengths, mbq, int(chunk_size),
                               _type_args(bam, B, mmq, wanted, ref_index))
            if err is not None:
                raise err
            # split references: every rank's histogram summed into the owner's (RCCL reduce over
            # xGMI, in rank 0's reference order on every rank), then kernel 2 on the owner
            for ref in ref_order:
                if ref not in split or ctx is None:
                    continue
                L = int(reference_lengths[ref])
                buf = split_acc.pop(ref, None)
                if buf is None:
                    buf = ctx.alloc(max(16, 4 * ncols * L))
                    buf.zero()
                with _phase("reduce"):
                    _group.reduce_i32(buf, ncols * L, owner[ref])
                if owner[ref] == _group.rank:
                    results[ref] = _finish_reference(ctx, buf, L, ncols, k, nf, nf2, _mode, tiles_of(ref),
                                                     _tiles is not None, scratch)
                else:
                    ctx.sync()
                    buf.free()
        finally:
            for b in split_acc.values():
                b.free()
        out = {}
        for ref in mine:
            n = nreads[ref]
            if _mode == "rows":
                out[ref] = {"rows": Rows(ref, results[ref], long_format), "num_reads": n}
            else:
                out[ref] = {"summary": results[ref], "num_reads": n,
                            "length": int(reference_lengths[ref])}
        if _group is not None:
            return out, owner, ref_order
        return out
    finally:
        _release(stream)


def _merge_shards(group, fl: _Faults, miss: bool, n_accepted: int, ref_order, names, nreads) -> bool:
    """Sharded decode: turn this rank's range-local fault ordinals into the file's (each range
    starts after the accepted reads of the ranges before it) and give every rank the faults the
    whole file holds, as one process streaming it would have recorded them.  False (on every rank)
    if any rank's range missed."""
    stopped = fl.inloop() is not None  # this range stopped at its first in-loop fault
    vals = [0 if miss else 1, int(stopped), fl.n_records, n_accepted,
            fl.keyerror[0] if fl.keyerror else -1,
            names.index(fl.keyerror[1]) if fl.keyerror and fl.keyerror[1] in names else -1,
            fl.clip if fl.clip is not None else -1]
    for r in ref_order:
        rg = fl.range_.get(r, (-1, -1))
        vals += [fl.type_ord.get(r, -1), rg[0], rg[1], nreads[r]]
    alls = group.all_gather_ints(vals)
    if any(v[0] == 0 for v in alls):
        return False
    # a range that stopped at an in-loop fault counted only part of its reads: the ranges after
    # it hold only later faults, which cannot change what is raised first
    cut = next((i for i, v in enumerate(alls) if v[1]), len(alls) - 1)
    bases = [0]
    for v in alls[:-1]:
        bases.append(bases[-1] + v[3])
    fl.n_records = sum(v[2] for v in alls)
    fl.keyerror = fl.clip = None
    fl.type_ord, fl.range_ = {}, {}
    for i in range(cut + 1):
        v, b = alls[i], bases[i]
        if v[4] >= 0 and fl.keyerror is None:
            fl.keyerror = (b + v[4], names[v[5]] if v[5] >= 0 else None)
        if v[6] >= 0 and fl.clip is None:
            fl.clip = b + v[6]
    # a reference's reads lie in its owner's range, or, split over ranks, in several: the first
    # fault is the smallest file ordinal over them, the read count their sum
    for j, r in enumerate(ref_order):
        nreads[r] = sum(v[7 + 4 * j + 3] for v in alls)
        for i in range(cut + 1):
            v = alls[i]
            if v[7 + 4 * j] >= 0:
                o = bases[i] + v[7 + 4 * j]
                fl.type_ord[r] = min(fl.type_ord.get(r, o), o)
            if v[7 + 4 * j + 1] >= 0:
                o = bases[i] + v[7 + 4 * j + 1]
                if r not in fl.range_ or o < fl.range_[r][0]:
                    fl.range_[r] = (o, v[7 + 4 * j + 2])
    return True


def _no_reads() -> D.BcReads:
    r = D.BcReads()
    r.sorted = 1
    r.seq_layout = D.BC_SEQ_EVENT
    return r


def _indexed(ctx, reads: D.BcReads, L: int, scratch: _Scratch) -> D.BcReads:
    """The slice as the fast kernels take it: an unsorted slice is first put in start order on
    the device (bc_reads_sort, into the reusable scratch).  No device index is built: a batch the
    CLI counts once never recovers it (bench.py, driver-clock figures: C3's run records cost
    k_index_runs ~19 us against ~12 us saved in k_rc; C2's tile index k_index_tiles ~6 us
    against ~0.8 us saved in k_pileup, whose tile groups then search pos[] themselves)."""
    if not reads.sorted and reads.n_reads > 1:
        nb = ctx.sort_bytes(reads)
        mem = scratch.get("sorted", nb).ptr
        scratch.pending_sort = (reads, mem)  # checked after the kernels (stream-ordered sort)
        reads = ctx.sort(reads, mem, nb, check_flags=False)
    return reads


def _device_reference(ctx, reads, L, mbq, ncols, k, nf, nf2, mode, tiles, want_tiles=False, scratch=None):
    """Kernel 1 + kernel 2 (+ reductions) for one reference whose reads are all in ``reads``;
    returns (result, first bad read of the batch).

    Coordinate-sorted batches take the fused pileup (bc_pileup / bc_pileup_summary); others
    count with the event-parallel kernel (bc_count) and then run kernel 2 (bc_stats)."""
    if L == 0:
        if reads.n_reads > 0:
            hist = ctx.alloc(4 * ncols)
            hist.zero()
            ctx.count(reads, 0, mbq, ncols, hist.ptr)
        bad = ctx.range_error()
        return _empty(k, mode), bad
    scratch = scratch or _Scratch(ctx)
    if reads.sorted and mode != "rows" and not want_tiles:
        # --summarise (main.py:469-499 prints six numbers per reference): the summary-only sweep
        # writes no per-position output, only numpy's buffer partials (bc_pileup_summary)
        work, dout = scratch.get("work", D.summary_work_bytes(L)), scratch.get("dout", 32)
        ctx.pileup_summary(reads, L, mbq, k, nf, nf2, None, None, None, None, None, work.ptr, dout.ptr)
        bad = ctx.range_error()
        s = dout.download(np.float64, 4)
        return {"L": L, "avg_cov": np.float64(s[0]), "avg_ent": np.float64(s[1]), "nnz": int(s[2])}, bad
    outs = scratch.outputs(k, L, want_pc=(mode == "rows"))
    hist = scratch.get("hist", 4 * ncols * L)
    pc_ptr = outs["pc"].ptr if outs["pc"] else None
    if reads.sorted and mode != "rows" and tiles:
        # --summarise-with-bed: pileup, summary and every amplicon window in one library call (a
        # deep batch's tail after kernel 1: kernel 2 + one launch)
        work, dout = scratch.get("work", D.summary_work_bytes(L)), scratch.get("dout", 32)
        lo = np.ascontiguousarray([a for a, _ in tiles], np.int64)
        hi = np.ascontiguousarray([b for _, b in tiles], np.int64)
        d_lo = scratch.get("amp_lo", lo.nbytes).upload(lo)
        d_hi = scratch.get("amp_hi", hi.nbytes).upload(hi)
        d_amp = scratch.get("amp", 48 * len(tiles))
        ctx.pileup_summary_amplicons(reads, L, mbq, k, nf, nf2, hist.ptr, outs["cov"].ptr, outs["ent"].ptr,
                                     outs["sec"].ptr, work.ptr, dout.ptr, d_lo.ptr, d_hi.ptr, len(tiles), d_amp.ptr)
        bad = ctx.range_error()
        s = dout.download(np.float64, 4)
        amp = d_amp.download(np.float64, 6 * len(tiles)).reshape(-1, 6)
        empty = [max(a, 0) > min(b, L - 1) for a, b in tiles]
        return {"L": L, "avg_cov": np.float64(s[0]), "avg_ent": np.float64(s[1]), "nnz": int(s[2]),
                "amplicons": (amp, empty)}, bad
    if reads.sorted and mode != "rows":
        # pileup + summary: the sparse sweep computes numpy's buffer partials in registers
        work, dout = scratch.get("work", D.summary_work_bytes(L)), scratch.get("dout", 32)
        ctx.pileup_summary(reads, L, mbq, k, nf, nf2, hist.ptr, outs["cov"].ptr, pc_ptr,
                           outs["ent"].ptr, outs["sec"].ptr, work.ptr, dout.ptr)
        bad = ctx.range_error()
        return _collect(ctx, outs, hist, L, k, ncols, mode, tiles, want_tiles, scratch, summarised=True), bad
    if reads.sorted:
        ctx.pileup(reads, L, mbq, k, nf, nf2, hist.ptr, outs["cov"].ptr, pc_ptr, outs["ent"].ptr,
                   outs["sec"].ptr)
        bad = ctx.range_error()
        return _collect(ctx, outs, hist, L, k, ncols, mode, tiles, want_tiles, scratch, stats_done=True), bad
    hist.zero(4 * ncols * L)
    ctx.count(reads, L, mbq, ncols, hist.ptr)
    bad = ctx.range_error()
    return _collect(ctx, outs, hist, L, k, ncols, mode, tiles, want_tiles, scratch), bad


def _finish_reference(ctx, acc, L, ncols, k, nf, nf2, mode, tiles, want_tiles, scratch):
    """Kernel 2 (+ reductions) for a reference whose counts were accumulated batch by batch in
    the device histogram ``acc`` (freed here)."""
    try:
        if L == 0:
            return _empty(k, mode)
        outs = scratch.outputs(k, L, want_pc=(mode == "rows"))
        return _collect(ctx, outs, acc, L, k, ncols, mode, tiles, want_tiles, scratch, nf=nf, nf2=nf2)
    finally:
        ctx.sync()
        acc.free()


def _empty(k, mode):
    if mode != "rows":
        return {"L": 0}
    return RefData(np.zeros((k, 0), np.int32), np.zeros((k, 0)), np.zeros(0), np.zeros(0), np.zeros(0, np.int32))


def _collect(ctx, outs, hist, L, k, ncols, mode, tiles, want_tiles, scratch, stats_done=False,
             summarised=False, nf=None, nf2=None):
    """The per-position statistics of the counts in ``hist`` (kernel 2, unless the fused pileup
    already ran it), then either the rows (downloaded) or the summary and amplicon reductions."""
    pc_ptr = outs["pc"].ptr if outs["pc"] else None
    if not (stats_done or summarised):
        if nf is None:
            nf, nf2 = norm_factors(k)
        ctx.stats(hist.ptr, L, k, nf, nf2, outs["cov"].ptr, pc_ptr, outs["ent"].ptr, outs["sec"].ptr)
    if mode == "rows":
        counts = hist.download(np.int32, ncols * L).reshape(ncols, L)
        return _download(outs, counts, k, L)
    dout = scratch.get("dout", 32)
    if not summarised:
        work = scratch.get("work", D.summary_work_bytes(L))
        ctx.summary(outs["cov"].ptr, outs["ent"].ptr, L, work.ptr, dout.ptr)
    res = {"L": L}
    s = dout.download(np.float64, 4)
    res.update(avg_cov=np.float64(s[0]), avg_ent=np.float64(s[1]), nnz=int(s[2]))
    if tiles is not None and len(tiles):
        lo = np.ascontiguousarray([a for a, _ in tiles], np.int64)
        hi = np.ascontiguousarray([b for _, b in tiles], np.int64)
        d_lo = ctx.alloc(lo.nbytes).upload(lo)
        d_hi = ctx.alloc(hi.nbytes).upload(hi)
        d_amp = ctx.alloc(48 * len(tiles))
        ctx.amplicons(outs["cov"].ptr, outs["ent"].ptr, outs["sec"].ptr, L, d_lo.ptr, d_hi.ptr,
                      len(tiles), d_amp.ptr)
        amp = d_amp.download(np.float64, 6 * len(tiles)).reshape(-1, 6)
        empty = [max(a, 0) > min(b, L - 1) for a, b in tiles]
        res["amplicons"] = (amp, empty)
    elif want_tiles:
        res["amplicons"] = (np.zeros((0, 6)), [])
    return res


class BaseCount:
    """main.py:208-359."""

    def __init__(self, bam, references=None, min_base_quality=0, min_mapping_quality=0,
                 chunk_size=1000000, show_n_bases=False, long_format=False, *, device=None,
                 _mode="rows", _tiles=None):
        self.columns = _columns(show_n_bases, long_format)
        self.data = get_basecounts(bam, references=references, min_base_quality=min_base_quality,
                                   min_mapping_quality=min_mapping_quality, chunk_size=chunk_size,
                                   show_n_bases=show_n_bases, long_format=long_format,
                                   device=device, _mode=_mode, _tiles=_tiles)
        self.references = list(self.data.keys())
        if _mode == "rows":
            self.reference_lengths = {ref: len(self.data[ref]["rows"]) for ref in self.references}
        else:
            self.reference_lengths = {ref: self.data[ref]["length"] for ref in self.references}

    def _check(self, reference):
        if self.data.get(reference) is None:
            raise Exception(f"{reference} is not a valid reference")

    def rows(self, reference=None):
        if reference is None:
            for ref in self.data.keys():
                yield from self.data[ref]["rows"]
        else:
            self._check(reference)
            yield from self.data[reference]["rows"]

    def records(self, reference=None):
        refs = list(self.data.keys()) if reference is None else [reference]
        if reference is not None:
            self._check(reference)
        for ref in refs:
            for row in self.data[ref]["rows"]:
                yield dict(zip(self.columns, row))

    def num_reads(self, reference=None):
        if reference is None:
            return sum([self.data[ref]["num_reads"] for ref in self.references])
        self._check(reference)
        return self.data[reference]["num_reads"]

    def _arrays(self, reference):
        refs = self.references if reference is None else [reference]
        if reference is not None:
            self._check(reference)
        return [self.data[r]["rows"] for r in refs]

    def mean_coverage(self, reference=None):
        """np.mean over every row's coverage (long format repeats each position k times)."""
        covs = []
        for rows in self._arrays(reference):
            c = rows.d.cov.astype(np.int64)
            covs.append(np.repeat(c, rows.k) if rows.long else c)
        return np.mean(np.concatenate(covs) if covs else np.zeros(0, np.int64))

    def mean_entropy(self, reference=None, min_coverage=0):
        ents = []
        for rows in self._arrays(reference):
            c = rows.d.cov.astype(np.int64)
            e = rows.d.ent
            if rows.long:
                c, e = np.repeat(c, rows.k), np.repeat(e, rows.k)
            ents.append(e[c >= min_coverage])
        if not ents:
            return np.mean([])
        allv = np.concatenate(ents)
        # an all-zero-coverage selection holds only int 1s in the reference: same mean
        return np.mean(allv)


def handle_arg(arg, name, default=None, provided_once=False):
    """main.py:362-375."""
    if arg is None:
        return default
    if provided_once:
        if len(arg) > 1:
            raise Exception(f"Argument --{name} can only be provided once")
        return arg[0]
    return list({a for a_list in arg for a in a_list})


def build_parser() -> argparse.ArgumentParser:
    """main.py:379-431, verbatim flags and help text."""
    parser = argparse.ArgumentParser(prog="basecount")
    parser.add_argument("bam", help="Path to BAM file (an index file is not required)")
    parser.add_argument("-v", "--version", action="version", version=__version__)
    parser.add_argument("--references", default=None, nargs="+", action="append",
                        help="Choose specific reference(s) to run basecount on")
    parser.add_argument("--min-base-quality", default=None, action="append",
                        help="Default value: 0")
    parser.add_argument("--min-mapping-quality", default=None, action="append",
                        help="Default value: 0")
    parser.add_argument("--chunk-size", default=None, action="append",
                        help="Max number of reads loaded into memory and basecounted at a given "
                             "time. Default value: 1000000")
    parser.add_argument("--show-n-bases", default=False, action="store_true",
                        help="Show counts of 'N' bases from reads, and include them in statistics")
    group = parser.add_mutually_exclusive_group()
    group.add_argument("--long-format", default=False, action="store_true",
                       help="Output per-position statistics in long format, instead of the "
                            "default wide format")
    group.add_argument("--summarise", default=False, action="store_true",
                       help="Output summary statistics")
    group.add_argument("--summarise-with-bed", default=None, action="append", metavar="BED_FILE",
                       help="Output summary statistics and amplicon vectors (calculated using the "
                            "provided BED file)")
    parser.add_argument("--decimal-places", default=None, action="append",
                        help="Default value: 3")
    return parser


def _np_round_str(x, dp):
    return str(round(x, dp))


def _columns(show_n_bases: bool, long_format: bool) -> list:
    """main.py:233-264."""
    if long_format:
        return ["reference", "position", "coverage", "base", "count", "percentage", "entropy",
                "secondary_entropy"]
    cols = ["reference", "position", "coverage", "num_a", "num_c", "num_g", "num_t", "num_ds",
            "num_n", "pc_a", "pc_c", "pc_g", "pc_t", "pc_ds", "pc_n", "entropy", "secondary_entropy"]
    if not show_n_bases:
        cols.pop(cols.index("num_n"))
        cols.pop(cols.index("pc_n"))
    return cols


_AMP_NAMES = ["mean_coverage_amplicon_vector", "median_coverage_amplicon_vector",
              "mean_entropy_amplicon_vector", "median_entropy_amplicon_vector",
              "mean_secondary_entropy_amplicon_vector", "median_secondary_entropy_amplicon_vector"]


def _print_summary(ref, s, ref_length, num_reads, dp, bed, bed_error):
    """main.py:469-595 for one reference (summary lines, then the amplicon vectors)."""
    if ref_length == 0:
        np.mean([])  # the reference's RuntimeWarning, then its ZeroDivisionError
        raise ZeroDivisionError("division by zero")
    pc_ref_coverage = 100 * (s["nnz"] / ref_length)
    summary_stats = {
        "reference_name": ref,
        "reference_length": round(ref_length, dp),
        "num_reads": round(num_reads, dp),
        "pc_reference_coverage": round(pc_ref_coverage, dp),
        "avg_depth": round(s["avg_cov"], dp),
        "avg_entropy": round(s["avg_ent"], dp),
    }
    for name, val in summary_stats.items():
        print(name, val, sep="\t")
    if bed is not None:
        if bed_error is not None:
            raise bed_error
        amp, empty = s["amplicons"]
        vecs = [[] for _ in range(6)]
        for i, e in enumerate(empty):
            for j in range(6):
                vecs[j].append(-1 if e else np.float64(amp[i, j]))
        for name, vec in zip(_AMP_NAMES, vecs):
            val = ", ".join([_np_round_str(x, dp) for x in vec]) if vec else "-"
            print(name, val, sep="\t")


def run(argv=None):
    """main.py:378-595: `basecount BAM [--long-format | --summarise | --summarise-with-bed BED]`.

    Under torchrun (WORLD_SIZE > 1) the references are sharded over the ranks (dist.py); the
    output is identical to a single process's."""
    args = build_parser().parse_args(argv)
    references = handle_arg(args.references, "references")
    min_base_quality = int(handle_arg(args.min_base_quality, "min-base-quality", default=0,
                                      provided_once=True))
    min_mapping_quality = int(handle_arg(args.min_mapping_quality, "min-mapping-quality",
                                         default=0, provided_once=True))
    chunk_size = int(handle_arg(args.chunk_size, "chunk-size", default=1000000,
                                provided_once=True))
    bed = handle_arg(args.summarise_with_bed, "bed", provided_once=True)
    decimal_places = int(handle_arg(args.decimal_places, "decimal_places", default=3,
                                    provided_once=True))
    from . import dist

    try:
        group = dist.Group() if dist.env()[0] > 1 else None  # RCCL (default) or gloo, DESIGN.md §6
    except dist.CommInitAbandoned as e:
        # an init thread is still blocked inside RCCL on some rank: nothing may run after it in
        # this process (not even interpreter shutdown's library teardown), on any rank
        print(f"basecount: {e}", file=sys.stderr, flush=True)
        os._exit(3)
    timing = os.environ.get("BASECOUNT_HIP_TIMING") not in (None, "", "0")
    t0 = None
    if timing:  # per-kernel device times and the wall time on stderr; stdout unchanged
        import time

        t0 = time.perf_counter()
        context().timing(True)
    global _DEFERRED
    _DEFERRED = []
    try:
        _run(args, references, min_base_quality, min_mapping_quality, chunk_size, bed,
             decimal_places, group)
    finally:
        deferred, _DEFERRED = _DEFERRED, None
        for h in deferred:
            h.close()
        if group is not None:
            group.close()
        if timing:
            _timing_report(time.perf_counter() - t0)


def _timing_report(wall_s: float) -> None:
    """BASECOUNT_HIP_TIMING=1: one stderr line per kernel id (launches, mean device time) and the
    run's wall time."""
    import sys

    try:
        rep = context().timing_report()
    except Exception as e:  # noqa: BLE001 - reporting must not mask the run's own outcome
        rep = {"error": str(e)}
    rank = os.environ.get("RANK", "0")
    for name, v in sorted(rep.items()):
        if isinstance(v, tuple):
            print(f"basecount[{rank}] kernel {name}: {v[0]} launches, {v[1]:.2f} us mean", file=sys.stderr)
    for name, v in PHASES.items():
        print(f"basecount[{rank}] host {name}: {v * 1e3:.2f} ms", file=sys.stderr)
    print(f"basecount[{rank}] wall {wall_s * 1e3:.2f} ms", file=sys.stderr)


def _run(args, references, min_base_quality, min_mapping_quality, chunk_size, bed, dp, group):
    from . import dist

    kw = dict(references=references, min_base_quality=min_base_quality,
              min_mapping_quality=min_mapping_quality, chunk_size=chunk_size,
              show_n_bases=args.show_n_bases, long_format=args.long_format)
    if (not args.summarise) and (bed is None):
        if group is None:
            bc = BaseCount(args.bam, **kw)
            print("\t".join(bc.columns))
            with _phase("format + write"):
                for ref in bc.references:
                    rows = bc.data[ref]["rows"]
                    d = rows.d
                    fmt.write_bytes(fmt.rows_text(ref, d.counts[: rows.k], d.pc, d.ent, d.sec, dp,
                                                  rows.long))
            return
        out, owner, order = get_basecounts(args.bam, **kw, _group=group)
        if group.rank == 0:
            print("\t".join(_columns(args.show_n_bases, args.long_format)), flush=True)
        group.barrier()
        blocks = {}
        for ref, v in out.items():
            rows = v["rows"]
            d = rows.d
            blocks[ref] = fmt.rows_text(ref, d.counts[: rows.k], d.pc, d.ent, d.sec, dp, rows.long)
        dist.ordered_write(group, order, owner, blocks, write=fmt.write_bytes)
        return

    bed_errors = {}

    def tiles(ref):
        # the reference re-parses the BED for every reference (main.py:502), after printing that
        # reference's summary: a bad BED is re-raised at that point of the output below
        try:
            scheme = load_scheme(bed)
        except Exception as e:  # noqa: BLE001 - re-raised in output order
            bed_errors[ref] = e
            return None
        return [(t[2]["inside_start"], t[2]["inside_end"]) for t in scheme]

    tk = dict(_mode="summary", _tiles=tiles if bed is not None else None)
    if group is None:
        bc = BaseCount(args.bam, **kw, **tk)
        for ref in bc.references:
            _print_summary(ref, bc.data[ref]["summary"], bc.reference_lengths[ref], bc.num_reads(ref),
                           dp, bed, bed_errors.get(ref))
        return
    # one process per GPU: exact numbers of the owned references gathered to rank 0 (float
    # repr round-trips), printed there in the reference's order
    out, owner, order = get_basecounts(args.bam, **kw, **tk, _group=group)
    payload = {}
    for ref, v in out.items():
        s = v["summary"]
        e = {"L": v["length"], "n": v["num_reads"]}
        if v["length"]:
            e.update(avg_cov=float(s["avg_cov"]), avg_ent=float(s["avg_ent"]), nnz=int(s["nnz"]))
            if "amplicons" in s:
                amp, empty = s["amplicons"]
                e.update(amp=np.asarray(amp, np.float64).tolist(), empty=[bool(x) for x in empty])
        payload[ref] = e
    parts = group.gather_bytes(json.dumps(payload).encode())
    if group.rank != 0:
        return
    merged = {}
    for part in parts:
        merged.update(json.loads(part.decode()))
    for ref in order:
        e = merged[ref]
        s = {}
        if e["L"]:
            s = {"avg_cov": np.float64(e["avg_cov"]), "avg_ent": np.float64(e["avg_ent"]), "nnz": e["nnz"]}
            if "amp" in e:
                s["amplicons"] = (np.asarray(e["amp"], np.float64).reshape(-1, 6), e["empty"])
        if bed is not None and owner[ref] != 0:
            tiles(ref)  # the BED errors of references computed elsewhere, evaluated here
        _print_summary(ref, s, e["L"], e["n"], dp, bed, bed_errors.get(ref))


if __name__ == "__main__":
    run()
