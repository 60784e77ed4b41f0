"""ctypes bindings for ``libbasecount_hip.so`` (``include/basecount_hip.h``).

``Context`` wraps one ``bc_ctx`` (device + stream); ``DeviceBuffer`` is a library-owned HBM
allocation; ``DeviceReads`` is an uploaded read batch (``bc_reads``).  Pointers may also come
from another allocator (e.g. ``torch.Tensor.data_ptr()``) — the C-ABI only sees addresses.

There is no CPU fallback: if the library or a gfx950 device is missing, the calls raise.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._native import _libs, _load

BC_E_ARG, BC_E_HIP, BC_E_RANGE, BC_E_NODEV, BC_E_COMM = -1, -2, -3, -4, -5
COMM_ID_BYTES = 128  # BC_COMM_ID_BYTES
BC_SEQ_BAM, BC_SEQ_EVENT = 0, 1
SHAPES = {"auto": 0, "tile": 1, "rc": 2, "tile_no_solo": 3}  # BC_SHAPE_*
KERNEL_NAMES = ("count", "stats", "rc", "pileup", "summary", "amplicons", "index", "solo", "sort")  # BC_K_* ids
BC_INDEX_RUNS, BC_INDEX_TILES, BC_INDEX_AUTO = 1, 2, 4
KERNEL_IDS = len(KERNEL_NAMES)


class BcReads(C.Structure):
    _fields_ = [
        ("n_reads", C.c_int64),
        ("pos", C.c_void_p),
        ("cig_beg", C.c_void_p),
        ("cig_n", C.c_void_p),
        ("seq_nib", C.c_void_p),
        ("cigar", C.c_void_p),
        ("n_cigar_words", C.c_int64),
        ("seq", C.c_void_p),
        ("seq_bytes", C.c_int64),
        ("qual", C.c_void_p),
        ("qual_bytes", C.c_int64),
        ("sorted", C.c_int32),
        ("max_span", C.c_int32),
        ("max_end", C.c_int64),
        ("seq_layout", C.c_int32),  # BC_SEQ_BAM 0 / BC_SEQ_EVENT 1
        ("run_chunks", C.c_int32),
        ("tile_reads", C.c_void_p),  # optional per-tile read ranges (bc_reads_upload)
        ("n_tiles", C.c_int64),
        ("read_runs", C.c_void_p),  # optional run records, 4 words per read (bc_reads_upload)
        ("index_tag", C.c_uint64),  # the batch the index was built for (0: none)
    ]


class BcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def lib() -> C.CDLL:
    L = _libs.get("libbasecount_hip.so")
    if L is not None:
        return L
    L = _load("libbasecount_hip.so")
    vp, i64, u32, dbl = C.c_void_p, C.c_int64, C.c_uint32, C.c_double
    sig = {
        "bc_last_error": ([], C.c_char_p),
        "bc_abi_version": ([], C.c_int),
        "bc_build_info": ([], C.c_char_p),
        "bc_device_count": ([C.POINTER(C.c_int)], C.c_int),
        "bc_ctx_create": ([C.c_int, vp, C.POINTER(vp)], C.c_int),
        "bc_ctx_destroy": ([vp], C.c_int),
        "bc_ctx_release_scratch": ([vp], C.c_int),
        "bc_ctx_stream": ([vp, C.POINTER(vp)], C.c_int),
        "bc_sync": ([vp], C.c_int),
        "bc_ctx_set_shape": ([vp, C.c_int, C.c_int, C.c_int], C.c_int),
        "bc_malloc": ([vp, C.c_size_t, C.POINTER(vp)], C.c_int),
        "bc_free": ([vp, vp], C.c_int),
        "bc_memcpy_h2d": ([vp, vp, vp, C.c_size_t], C.c_int),
        "bc_memcpy_d2h": ([vp, vp, vp, C.c_size_t], C.c_int),
        "bc_memset": ([vp, vp, C.c_int, C.c_size_t], C.c_int),
        "bc_reads_upload": ([vp, C.POINTER(BcReads), C.POINTER(BcReads)], C.c_int),
        "bc_reads_free": ([vp, C.POINTER(BcReads)], C.c_int),
        "bc_reads_index_bytes": ([vp, C.POINTER(BcReads), i64, C.c_int, C.POINTER(C.c_size_t)], C.c_int),
        "bc_reads_index": ([vp, C.POINTER(BcReads), i64, C.c_int, vp, C.c_size_t], C.c_int),
        "bc_reads_sort_bytes": ([vp, C.POINTER(BcReads), C.POINTER(C.c_size_t)], C.c_int),
        "bc_reads_sort": ([vp, C.POINTER(BcReads), C.POINTER(BcReads), vp, C.c_size_t], C.c_int),
        "bc_reads_sort_check": ([vp, C.POINTER(BcReads), vp], C.c_int),
        "bc_count": ([vp, C.POINTER(BcReads), i64, u32, C.c_int, vp], C.c_int),
        "bc_range_error": ([vp, C.POINTER(i64)], C.c_int),
        "bc_stats": ([vp, vp, i64, C.c_int, dbl, dbl, vp, vp, vp, vp], C.c_int),
        "bc_summary_work_bytes": ([i64], C.c_size_t),
        "bc_seq_event_bytes": ([i64], C.c_size_t),
        "bc_seq_to_event": ([vp, vp, i64, vp], C.c_int),
        "bc_summary": ([vp, vp, vp, i64, vp, vp], C.c_int),
        "bc_amplicons": ([vp, vp, vp, vp, i64, vp, vp, C.c_int32, vp], C.c_int),
        "bc_pileup_summary_amplicons": ([vp, C.POINTER(BcReads), i64, u32, C.c_int, dbl, dbl, vp, vp, vp, vp, vp, vp,
                                         vp, vp, C.c_int32, vp], C.c_int),
        "bc_bcount_host": ([C.c_int, i64, u32, C.POINTER(BcReads), vp, C.POINTER(i64),
                            C.POINTER(i64)], C.c_int),
        "bc_pileup": ([vp, C.POINTER(BcReads), i64, u32, C.c_int, dbl, dbl, vp, vp, vp, vp, vp],
                      C.c_int),
        "bc_pileup_summary": ([vp, C.POINTER(BcReads), i64, u32, C.c_int, dbl, dbl, vp, vp, vp, vp, vp,
                               vp, vp], C.c_int),
        "bc_pileup_partials": ([vp, C.POINTER(BcReads), i64, u32, C.c_int, dbl, dbl, vp, vp, vp, vp, vp,
                                vp], C.c_int),
        "bc_summary_fold": ([vp, C.c_int, vp, vp, vp], C.c_int),
        "bc_graph_begin": ([vp], C.c_int),
        "bc_graph_end": ([vp, C.POINTER(vp)], C.c_int),
        "bc_graph_launch": ([vp, vp], C.c_int),
        "bc_graph_destroy": ([vp], C.c_int),
        "bc_timing_enable": ([vp, C.c_int], C.c_int),
        "bc_timing_report": ([vp, vp, vp], C.c_int),
        "bc_event_record": ([vp, C.c_int], C.c_int),
        "bc_ctx_wait": ([vp, vp], C.c_int),
        "bc_event_elapsed_ms": ([vp, C.c_int, C.c_int, C.POINTER(C.c_float)], C.c_int),
        # multi-GPU (bc_comm.hip)
        "bc_comm_unique_id": ([vp], C.c_int),
        "bc_comm_init": ([vp, vp, C.c_int, C.c_int, C.POINTER(vp)], C.c_int),
        "bc_comm_destroy": ([vp], C.c_int),
        "bc_comm_rank": ([vp, C.POINTER(C.c_int), C.POINTER(C.c_int)], C.c_int),
        "bc_comm_barrier": ([vp], C.c_int),
        "bc_allgather_i64": ([vp, vp, i64, vp], C.c_int),
        "bc_broadcast_bytes": ([vp, vp, i64, C.c_int], C.c_int),
        "bc_gather_layout": ([vp, C.c_int, vp], C.c_int),
        "bc_gather_bytes": ([vp, vp, i64, vp, vp, C.c_int], C.c_int),
        "bc_gather_dev": ([vp, vp, i64, vp, vp, C.c_int], C.c_int),
        "bc_reduce_i32_dev": ([vp, vp, vp, i64, C.c_int], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return L


def check(rc: int) -> None:
    if rc != 0:
        raise BcError(rc, lib().bc_last_error().decode(errors="replace"))


def build_info() -> str:
    """bc_build_info(): e.g. "gfx950 diag=0 phase_trace=0"."""
    return lib().bc_build_info().decode()


def device_count() -> int:
    n = C.c_int(0)
    check(lib().bc_device_count(C.byref(n)))
    return n.value


class DeviceBuffer:
    """Library-owned HBM allocation."""

    def __init__(self, ctx: "Context", nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(lib().bc_malloc(ctx.h, self.nbytes, C.byref(p)))
        self.ptr = p.value

    def free(self):
        if self.ptr:
            check(lib().bc_free(self.ctx.h, self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def upload(self, arr: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes
        check(lib().bc_memcpy_h2d(self.ctx.h, self.ptr, a.ctypes.data, a.nbytes))
        self.ctx._keep.append(a)  # keep host staging alive until the next sync
        return self

    def download(self, dtype, count: int, offset_bytes: int = 0) -> np.ndarray:
        out = np.empty(int(count), dtype)
        if out.nbytes:
            check(lib().bc_memcpy_d2h(self.ctx.h, out.ctypes.data, self.ptr + offset_bytes,
                                      out.nbytes))
            self.ctx.sync()
        return out

    def zero(self, nbytes: int | None = None):
        check(lib().bc_memset(self.ctx.h, self.ptr, 0, self.nbytes if nbytes is None else nbytes))


def host_reads(b: dict) -> tuple:
    """bc_reads over host numpy arrays (keeps the arrays referenced in the returned tuple)."""
    keep = {}
    for k, dt in (("pos", np.int32), ("cig_beg", np.uint32), ("cig_n", np.uint32),
                  ("seq_nib", np.uint32), ("cigar", np.uint32), ("seq", np.uint8)):
        keep[k] = np.ascontiguousarray(b[k], dt)
    q = b.get("qual")
    keep["qual"] = None if q is None else np.ascontiguousarray(q, np.uint8)
    r = BcReads()
    r.n_reads = keep["pos"].size
    for k in ("pos", "cig_beg", "cig_n", "seq_nib", "cigar", "seq"):
        setattr(r, k, keep[k].ctypes.data if keep[k].size else None)
    r.n_cigar_words = keep["cigar"].size
    r.seq_bytes = keep["seq"].size
    if keep["qual"] is not None:
        r.qual = keep["qual"].ctypes.data if keep["qual"].size else None
        r.qual_bytes = keep["qual"].size
    r.sorted = int(b.get("sorted", 0))
    r.max_span = int(b.get("max_span", 0))
    if b.get("seq_event") is not None:
        # the host already holds the kernels' layout (bcio decoder / bam.seq_to_event): sent as
        # is, no device conversion pass
        keep["seq"] = np.ascontiguousarray(b["seq_event"], np.uint8)
        r.seq = keep["seq"].ctypes.data
        r.seq_layout = BC_SEQ_EVENT
    return r, keep


class DeviceReads:
    """A read batch resident in HBM (library-owned copy of a host batch)."""

    def __init__(self, ctx: "Context", b: dict):
        self.ctx = ctx
        hr, keep = host_reads(b)
        self.r = BcReads()
        check(lib().bc_reads_upload(ctx.h, C.byref(hr), C.byref(self.r)))
        self.n = int(self.r.n_reads)

    def free(self):
        if getattr(self, "r", None) is not None and self.ctx.h:
            check(lib().bc_reads_free(self.ctx.h, C.byref(self.r)))
            self.r = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Context:
    def __init__(self, device: int = 0, stream: int | None = None):
        self.device = int(device)
        h = C.c_void_p()
        check(lib().bc_ctx_create(self.device, stream, C.byref(h)))
        self.h = h.value
        self._keep = []

    def close(self):
        if self.h:
            lib().bc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def release_scratch(self) -> None:
        """bc_ctx_release_scratch: the context's own grow-only device scratch given back."""
        check(lib().bc_ctx_release_scratch(self.h))

    def set_shape(self, shape: str = "auto", tile_waves: int = 0, reads_per_block: int = 0) -> None:
        """Kernel-shape override for bc_count / bc_pileup (bc_ctx_set_shape): "auto", "tile",
        "rc" or "tile_no_solo"; tile_waves 0/1/2/4/8; reads_per_block 0 or 1..32768."""
        check(lib().bc_ctx_set_shape(self.h, SHAPES[shape], int(tile_waves), int(reads_per_block)))

    def sync(self):
        check(lib().bc_sync(self.h))
        self._keep.clear()

    def stream(self) -> int:
        s = C.c_void_p()
        check(lib().bc_ctx_stream(self.h, C.byref(s)))
        return s.value or 0

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    # kernels ---------------------------------------------------------------------------
    def count(self, reads, ref_len: int, mbq: int, ncols: int, d_hist: int) -> None:
        r = reads.r if isinstance(reads, DeviceReads) else reads
        check(lib().bc_count(self.h, C.byref(r), int(ref_len), int(mbq), int(ncols), d_hist))

    def index_bytes(self, reads, L: int, what: int = BC_INDEX_AUTO) -> int:
        """bc_reads_index_bytes: device bytes the batch's index needs (0: nothing to build)."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        n = C.c_size_t(0)
        check(lib().bc_reads_index_bytes(self.h, C.byref(r), int(L), int(what), C.byref(n)))
        return int(n.value)

    def index(self, reads, L: int, d_mem, nbytes: int, what: int = BC_INDEX_AUTO) -> None:
        """bc_reads_index: build the batch's device index (run records / chunk summaries / tile
        index) into d_mem on the stream and set the index fields of the bc_reads in place."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        check(lib().bc_reads_index(self.h, C.byref(r), int(L), int(what), d_mem, int(nbytes)))

    def sort_bytes(self, reads) -> int:
        """bc_reads_sort_bytes: device bytes the sorted copy of an unsorted batch needs."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        n = C.c_size_t(0)
        check(lib().bc_reads_sort_bytes(self.h, C.byref(r), C.byref(n)))
        return int(n.value)

    def sort(self, reads, d_mem, nbytes: int, check_flags: bool = True) -> BcReads:
        """bc_reads_sort: a coordinate-sorted copy of the batch, built on the device into d_mem
        (stream-ordered: the call only enqueues); returns its bc_reads (no index yet).  With
        ``check_flags`` the device's error flags are read at once (sort_check, a sync); without it the
        caller runs sort_check(reads, d_mem) later, e.g. after the batch's kernels."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        out = BcReads()
        check(lib().bc_reads_sort(self.h, C.byref(r), C.byref(out), d_mem, int(nbytes)))
        if check_flags:
            self.sort_check(r, d_mem)
        return out

    def sort_check(self, reads, d_mem) -> None:
        """bc_reads_sort_check: waits for the stream, raises BcError (BC_E_ARG) if the sort of
        ``reads`` into d_mem saw a start outside [0, max_end] or overlapping sequences."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        check(lib().bc_reads_sort_check(self.h, C.byref(r), d_mem))

    def pileup(self, reads, L, mbq, k, nf, nf2, d_counts, d_cov, d_pc, d_ent, d_sec):
        """Fused kernel 1 + kernel 2 (bc_pileup) for a coordinate-sorted batch: one launch."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        check(lib().bc_pileup(self.h, C.byref(r), int(L), int(mbq), int(k), float(nf), float(nf2),
                              d_counts, d_cov, d_pc, d_ent, d_sec))

    def pileup_summary(self, reads, L, mbq, k, nf, nf2, d_counts, d_cov, d_pc, d_ent, d_sec, d_work,
                       d_out):
        """bc_pileup + bc_summary in one call (the sparse sweep computes the summary partials)."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        check(lib().bc_pileup_summary(self.h, C.byref(r), int(L), int(mbq), int(k), float(nf),
                                      float(nf2), d_counts, d_cov, d_pc, d_ent, d_sec, d_work, d_out))

    def pileup_partials(self, reads, L, mbq, k, nf, nf2, d_counts, d_cov, d_pc, d_ent, d_sec, d_work):
        """bc_pileup_partials: pileup + the summary's per-buffer partials (fold them with
        summary_fold)."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        check(lib().bc_pileup_partials(self.h, C.byref(r), int(L), int(mbq), int(k), float(nf),
                                       float(nf2), d_counts, d_cov, d_pc, d_ent, d_sec, d_work))

    def summary_fold(self, lens, works, outs) -> None:
        """bc_summary_fold over several references (device pointers works / outs)."""
        n = len(lens)
        la = (C.c_int64 * max(1, n))(*[int(x) for x in lens])
        wa = (C.c_void_p * max(1, n))(*works)
        oa = (C.c_void_p * max(1, n))(*outs)
        check(lib().bc_summary_fold(self.h, n, la, wa, oa))

    def capture(self, fn) -> "Graph":
        """Record the compute calls made by fn() into a hipGraph (replay with Graph.launch)."""
        check(lib().bc_graph_begin(self.h))
        try:
            fn()
        finally:
            g = C.c_void_p()
            rc = lib().bc_graph_end(self.h, C.byref(g))
        check(rc)
        return Graph(self, g.value)

    def timing(self, on: bool = True) -> None:
        check(lib().bc_timing_enable(self.h, int(bool(on))))

    def timing_report(self) -> dict:
        """{kernel: (launches, mean_us)} since the last report (synchronises)."""
        n = np.zeros(KERNEL_IDS, np.int64)
        us = np.zeros(KERNEL_IDS, np.float64)
        check(lib().bc_timing_report(self.h, n.ctypes.data, us.ctypes.data))
        return {name: (int(n[i]), float(us[i])) for i, name in enumerate(KERNEL_NAMES) if n[i]}

    def seq_to_event(self, d_bam: int, seq_bytes: int, d_event: int) -> None:
        """BAM-packed sequence -> BC_SEQ_EVENT (d_event may alias d_bam; it needs
        seq_event_bytes(seq_bytes) bytes)."""
        check(lib().bc_seq_to_event(self.h, d_bam, int(seq_bytes), d_event))

    def wait(self, other: "Context") -> None:
        """bc_ctx_wait: this context's later work waits for everything enqueued on `other`."""
        check(lib().bc_ctx_wait(self.h, other.h))

    def event_record(self, slot: int) -> None:
        """Record hipEvent `slot` on the context's stream (region timing)."""
        check(lib().bc_event_record(self.h, int(slot)))

    def event_elapsed_ms(self, slot0: int, slot1: int) -> float:
        ms = C.c_float(0.0)
        check(lib().bc_event_elapsed_ms(self.h, int(slot0), int(slot1), C.byref(ms)))
        return float(ms.value)

    def range_error(self) -> int:
        v = C.c_int64(-1)
        check(lib().bc_range_error(self.h, C.byref(v)))
        return v.value

    def stats(self, d_hist, L, k, nf, nf2, d_cov, d_pc, d_ent, d_sec) -> None:
        check(lib().bc_stats(self.h, d_hist, int(L), int(k), float(nf), float(nf2), d_cov, d_pc,
                             d_ent, d_sec))

    def summary(self, d_cov, d_ent, L, d_work, d_out) -> None:
        check(lib().bc_summary(self.h, d_cov, d_ent, int(L), d_work, d_out))

    def pileup_summary_amplicons(self, reads, L, mbq, k, nf, nf2, d_counts, d_cov, d_ent, d_sec, d_work, d_out,
                                 d_lo, d_hi, n_tiles, d_amp) -> None:
        """bc_pileup_summary_amplicons: --summarise-with-bed for one reference (the summary's 4
        doubles into d_out, 6 per amplicon window into d_amp); a deep batch's tail after kernel 1
        is kernel 2 + ONE launch."""
        r = reads.r if isinstance(reads, DeviceReads) else reads
        check(lib().bc_pileup_summary_amplicons(self.h, C.byref(r), int(L), int(mbq), int(k), float(nf), float(nf2),
                                                d_counts, d_cov, d_ent, d_sec, d_work, d_out, d_lo, d_hi,
                                                int(n_tiles), d_amp))

    def amplicons(self, d_cov, d_ent, d_sec, L, d_lo, d_hi, n_tiles, d_out) -> None:
        check(lib().bc_amplicons(self.h, d_cov, d_ent, d_sec, int(L), d_lo, d_hi, int(n_tiles),
                                 d_out))


class Graph:
    def __init__(self, ctx: Context, h: int):
        self.ctx, self.h = ctx, h

    def launch(self):
        check(lib().bc_graph_launch(self.ctx.h, self.h))

    def __del__(self):
        try:
            if self.h:
                lib().bc_graph_destroy(self.h)
                self.h = None
        except Exception:
            pass


def seq_event_bytes(seq_bytes: int) -> int:
    return int(lib().bc_seq_event_bytes(int(seq_bytes)))


def summary_work_bytes(L: int) -> int:
    return int(lib().bc_summary_work_bytes(int(L)))
