"""GPU parity: the HIP path (through the C-ABI) against the oracle and the reference's golden
fixtures.  Integer results must be bit-exact; entropies within 1e-6 (north_star), and the
printed text byte-identical."""
import gzip
import io
import os
import subprocess
import sys
import contextlib

import numpy as np
import pytest

import oracle as O
from basecount_amd import device as D
from basecount_amd import synth
from basecount_amd.main import norm_factors

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    return D.Context(0)


@pytest.fixture(autouse=True)
def _auto_shape(request):
    """Every test starts and ends with the automatic kernel shape (bc_ctx_set_shape)."""
    yield
    if "ctx" in request.fixturenames:
        request.getfixturevalue("ctx").set_shape("auto")


def gpu_count(ctx, b, L, mbq, ncols, **kw):
    b = dict(b, **kw)
    r = D.DeviceReads(ctx, b)
    hist = ctx.alloc(max(4, 4 * ncols * L))
    hist.zero()
    ctx.count(r, L, mbq, ncols, hist.ptr)
    bad = ctx.range_error()
    h = hist.download(np.int32, ncols * L).reshape(ncols, L)
    r.free()
    return h, bad


def random_batch(rng, L, n, long_skip=False, sort=True, nfrac=0.05, starts=None):
    """n random reads (mixed CIGARs, 5 % non-ACGT letters) on a reference of L positions, starts
    uniform (or drawn by ``starts(rng, span)``), coordinate-sorted unless ``sort`` is False."""
    pos, cigs, seqs, quals = [], [], [], []
    for _ in range(n):
        ops = []
        if rng.random() < 0.4:
            ops.append((4, int(rng.integers(1, 6))))
        ops.append((0, int(rng.integers(1, 60))))
        for _ in range(int(rng.integers(0, 5))):
            op = int(rng.choice([0, 1, 2, 3, 6, 7, 8, 9]))
            ln = int(rng.integers(1, 8))
            if op == 3 and long_skip and rng.random() < 0.3:
                ln = int(rng.integers(3000, 9000))
            ops.append((op, ln))
        ops.append((0, int(rng.integers(1, 60))))
        if rng.random() < 0.4:
            ops.append((4, int(rng.integers(1, 6))))
        span = sum(ln for op, ln in ops if op in (0, 2, 3, 7, 8))
        if span >= L:
            continue
        q = sum(ln for op, ln in ops if op in (0, 1, 4, 7, 8))
        codes = synth.ACGT[rng.integers(0, 4, q)]
        codes[rng.random(q) < nfrac] = rng.choice([15, 0, 5, 3])
        seqs.append(codes)
        quals.append(rng.integers(0, 45, q).astype(np.uint8))
        pos.append(int(rng.integers(0, L - span)) if starts is None else int(starts(rng, span)))
        cigs.append(ops)
    return build_batch(pos, cigs, seqs, quals, sort)


def build_batch(pos, cigs, seqs, quals, sort=True):
    """The batch dict of reads given as starts, CIGAR (op, len) lists, base codes and qualities."""
    order = np.argsort(pos, kind="stable") if sort else np.arange(len(pos))
    pos = [pos[i] for i in order]
    cigs = [cigs[i] for i in order]
    seqs = [seqs[i] for i in order]
    quals = [quals[i] for i in order]
    # BAM-like buffers: each read's SEQ starts on a byte boundary
    nib = np.zeros(len(pos) + 1, np.int64)
    nib[1:] = np.cumsum([len(s) + (len(s) & 1) for s in seqs])
    allc = np.zeros(int(nib[-1]) + 2, np.uint8)
    qual = np.zeros(int(nib[-1]) + 2, np.uint8)
    for i, (s, q) in enumerate(zip(seqs, quals)):
        allc[nib[i]: nib[i] + len(s)] = s
        qual[nib[i]: nib[i] + len(q)] = q
    seq = ((allc[0::2] << 4) | allc[1::2]).astype(np.uint8)
    cig_n = np.array([len(c) for c in cigs], np.uint32)
    cig_beg = np.zeros(len(cigs), np.uint32)
    cig_beg[1:] = np.cumsum(cig_n)[:-1]
    cigar = np.array([(ln << 4) | op for c in cigs for op, ln in c], np.uint32)
    qstart = np.array([c[0][1] if c[0][0] == 4 else 0 for c in cigs], np.int64)
    return dict(pos=np.array(pos, np.int32), cig_beg=cig_beg, cig_n=cig_n,
                seq_nib=(nib[:-1] + qstart).astype(np.uint32), cigar=cigar, seq=seq, qual=qual)


@pytest.mark.parametrize("seed,L,n,sort,long_skip", [
    (1, 500, 300, True, False), (2, 30_000, 20_000, True, False), (3, 2_000, 5_000, False, False),
    (4, 50_000, 3_000, True, True), (5, 300, 4_000, True, False), (6, 1_000_000, 2_000, True, False),
])
@pytest.mark.parametrize("mbq", [0, 20, 40])
@pytest.mark.parametrize("path", ["tile", "rc"])
def test_kernel1_matches_oracle(ctx, seed, L, n, sort, long_skip, mbq, path):
    """Sorted batches take the tiled (k_pileup) or the read-chunked (k_rc) kernel, unsorted
    ones the event-parallel k_count: identical counts."""
    ctx.set_shape(path)
    rng = np.random.default_rng(seed)
    b = random_batch(rng, L, n, long_skip=long_skip, sort=sort)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    for ncols in (5, 6):
        got, bad = gpu_count(ctx, b, L, mbq, ncols)
        assert bad == -1
        assert np.array_equal(got, exp[:, :ncols].T.astype(np.int32)), (seed, ncols)


def shaped_batch(rng, L, n, templates, nfrac=0.02):
    """Sorted reads whose CIGARs are drawn from `templates` (lists of (op, len)): targets the
    read-chunked kernel's event image (<= 2 runs from the read start to its end) and the shapes
    that make a chunk fall back to the run tables."""
    pos, cigs, seqs, quals = [], [], [], []
    for _ in range(n):
        ops = templates[int(rng.integers(0, len(templates)))]
        span = sum(ln for op, ln in ops if op in (0, 2, 3, 7, 8))
        q = sum(ln for op, ln in ops if op in (0, 1, 4, 7, 8))
        codes = synth.ACGT[rng.integers(0, 4, q)]
        codes[rng.random(q) < nfrac] = rng.choice([15, 0, 5, 3])
        seqs.append(codes)
        quals.append(rng.integers(0, 45, q).astype(np.uint8))
        pos.append(int(rng.integers(0, L - span)))
        cigs.append(ops)
    order = np.argsort(pos, kind="stable")
    pos, cigs = [pos[i] for i in order], [cigs[i] for i in order]
    seqs, quals = [seqs[i] for i in order], [quals[i] for i in order]
    nib = np.zeros(len(pos) + 1, np.int64)
    nib[1:] = np.cumsum([len(s) + (len(s) & 1) for s in seqs])
    allc = np.zeros(int(nib[-1]) + 2, np.uint8)
    qual = np.zeros(int(nib[-1]) + 2, np.uint8)
    for i, (s, q) in enumerate(zip(seqs, quals)):
        allc[nib[i]: nib[i] + len(s)] = s
        qual[nib[i]: nib[i] + len(q)] = q
    seq = ((allc[0::2] << 4) | allc[1::2]).astype(np.uint8)
    cig_n = np.array([len(c) for c in cigs], np.uint32)
    cig_beg = np.zeros(len(cigs), np.uint32)
    cig_beg[1:] = np.cumsum(cig_n)[:-1]
    cigar = np.array([(ln << 4) | op for c in cigs for op, ln in c], np.uint32)
    qstart = np.array([c[0][1] if c[0][0] == 4 else 0 for c in cigs], np.int64)
    return dict(pos=np.array(pos, np.int32), cig_beg=cig_beg, cig_n=cig_n,
                seq_nib=(nib[:-1] + qstart).astype(np.uint32), cigar=cigar, seq=seq, qual=qual)


IMAGE_OK = [[(0, 150)], [(4, 5), (0, 140), (4, 5)], [(0, 70), (2, 2), (0, 78)],
            [(0, 70), (1, 3), (0, 77)], [(0, 60), (3, 4), (0, 80)], [(0, 40), (7, 10), (8, 1), (0, 99)],
            [(5, 3), (0, 100), (2, 1), (0, 49), (4, 2)]]
FALLBACK = [[(2, 3), (0, 147)], [(0, 147), (2, 3)], [(0, 50), (2, 2), (0, 50), (2, 2), (0, 46)],
            [(0, 100), (3, 5000), (0, 50)], [(1, 4), (0, 146)]]
# 2 x 250 bp-style reads: a 256-read chunk's sequence (~32 KB) does not fit k_rc's stage, and
# every read is longer than a gather slot (such chunks keep the run-table walk)
LONG250 = [[(0, 250)], [(4, 5), (0, 240), (4, 5)], [(0, 120), (2, 2), (0, 130)], [(0, 100), (1, 2), (0, 148)]]


@pytest.mark.parametrize("mix", ["image", "fallback", "mixed", "long250"])
@pytest.mark.parametrize("mbq,ncols", [(0, 5), (20, 6)])
def test_rc_event_image_shapes(ctx, mix, mbq, ncols):
    """Deep sorted batches through k_rc: chunks the event image takes, chunks whose reads start
    or end with a deletion / have 3 runs / span too many windows (run tables), both mixed, and
    deep 250-base reads (chunks too long for the stage and the gather slots)."""
    ctx.set_shape("rc")
    tpl = {"image": IMAGE_OK, "fallback": FALLBACK, "mixed": IMAGE_OK + FALLBACK[:2], "long250": LONG250}[mix]
    rng = np.random.default_rng({"image": 31, "fallback": 32, "mixed": 33, "long250": 34}[mix])
    L = 12_000
    b = shaped_batch(rng, L, 40_000, tpl)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    got, bad = gpu_count(ctx, b, L, mbq, ncols)
    assert bad == -1
    assert np.array_equal(got, exp[:, :ncols].T.astype(np.int32)), mix


@pytest.mark.parametrize("mix", ["image", "fallback", "mixed"])
@pytest.mark.parametrize("mbq,k", [(0, 5), (20, 6)])
def test_rc_pileup_shapes(ctx, mix, mbq, k):
    """bc_pileup through k_rc + k_stats on image chunks (deferred flush), run-table chunks and
    complex reads: counts and statistics exact, and repeated calls show the context's
    accumulation scratch left zeroed."""
    ctx.set_shape("rc")
    tpl = {"image": IMAGE_OK, "fallback": FALLBACK, "mixed": IMAGE_OK + FALLBACK[:2]}[mix]
    rng = np.random.default_rng({"image": 41, "fallback": 42, "mixed": 43}[mix])
    L = 12_000
    b = shaped_batch(rng, L, 40_000, tpl)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    ocov, opc, oent, osec = O.stats(exp, k == 6)
    for rep in range(2):
        (cnt, cov, pc, ent, sec), bad = gpu_pileup(ctx, b, L, mbq, k)
        assert bad == -1
        assert np.array_equal(cnt, exp[:, :k].T.astype(np.int32)), (mix, rep)
        assert np.array_equal(cov, ocov) and np.array_equal(pc, opc)
        assert np.array_equal(ent, oent) and np.array_equal(sec, osec)


def test_rc_pileup_after_range_error(ctx):
    """A k_rc bc_pileup call with reads past the reference end: the first offending read, and
    the next call on the same context is exact (the scratch left zeroed)."""
    ctx.set_shape("rc")
    rng = np.random.default_rng(44)
    L = 5_000
    b = shaped_batch(rng, L + 400, 30_000, IMAGE_OK[:4])
    _, (br, _) = O.bcount(L, 0, b)
    assert br != -1
    _, bad = gpu_pileup(ctx, b, L, 0, 5)
    assert bad == br
    L2 = L + 400
    exp, (br2, _) = O.bcount(L2, 0, b)
    assert br2 == -1
    (cnt, cov, _, ent, _), bad2 = gpu_pileup(ctx, b, L2, 0, 5)
    assert bad2 == -1 and np.array_equal(cnt, exp[:, :5].T.astype(np.int32))
    ocov, _, oent, _ = O.stats(exp, False)
    assert np.array_equal(cov, ocov) and np.array_equal(ent, oent)


@pytest.mark.parametrize("mix", ["image", "fallback", "mixed"])
@pytest.mark.parametrize("mbq,ncols", [(0, 5), (0, 6), (20, 5)])
def test_rc_same_without_run_records(ctx, mix, mbq, ncols):
    """k_rc from the upload's run records (bc_reads.read_runs, the CIGARs decoded once on the
    host) and from its own CIGAR decode: identical counts and first out-of-range read."""
    ctx.set_shape("rc")
    tpl = {"image": IMAGE_OK, "fallback": FALLBACK, "mixed": IMAGE_OK + FALLBACK[:2]}[mix]
    rng = np.random.default_rng({"image": 51, "fallback": 52, "mixed": 53}[mix])
    L = 9_000
    b = shaped_batch(rng, L + 300, 30_000, tpl)
    for L2 in (L + 300, L):
        got = []
        for use in (True, False):
            r = D.DeviceReads(ctx, b)
            assert r.r.read_runs
            if not use:
                r.r.read_runs = None
            hist = ctx.alloc(4 * ncols * L2)
            hist.zero()
            ctx.count(r, L2, mbq, ncols, hist.ptr)
            got.append((ctx.range_error(), hist.download(np.int32, ncols * L2)))
            r.free()
        assert got[0][0] == got[1][0]
        assert np.array_equal(got[0][1], got[1][1])
        exp, (br, _) = O.bcount(L2, mbq, b)
        assert got[0][0] == br
        if br == -1:
            assert np.array_equal(got[0][1].reshape(ncols, L2), exp[:, :ncols].T.astype(np.int32))


IMAGE_DEEP = IMAGE_OK + [[(0, 50), (2, 20), (0, 80)], [(0, 40), (3, 41), (0, 60)],
                         [(4, 3), (0, 31), (2, 9), (0, 90), (4, 2)], [(0, 32), (2, 32), (0, 64)],
                         [(0, 1), (2, 100), (0, 1)], [(0, 8)], [(0, 63), (1, 9), (0, 64)]]


@pytest.mark.parametrize("mbq,ncols", [(0, 5), (0, 6), (20, 5)])
def test_rc_event_image_deep(ctx, mbq, ncols):
    """Deep batches whose 256-read chunks fit the event image (<= 23 windows): one- and two-run
    reads, deletions and reference skips that cover whole image rows, boundaries on and off
    the rows' 8-position edges; with the upload's run records and chunk summaries, with the
    records only, and from the CIGARs."""
    ctx.set_shape("rc")
    rng = np.random.default_rng(35 + mbq + ncols)
    L = 3_000
    b = shaped_batch(rng, L, 150_000, IMAGE_DEEP)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    for mode in ("records+summaries", "records", "cigars"):
        r = D.DeviceReads(ctx, b)
        assert r.r.read_runs and r.r.run_chunks > 0  # one per k_rc chunk of the batch
        if mode != "records+summaries":
            r.r.run_chunks = 0  # the block reduces the chunk bounds itself
        if mode == "cigars":
            r.r.read_runs = None
        hist = ctx.alloc(4 * ncols * L)
        hist.zero()
        ctx.count(r, L, mbq, ncols, hist.ptr)
        assert ctx.range_error() == -1
        got = hist.download(np.int32, ncols * L).reshape(ncols, L)
        r.free()
        assert np.array_equal(got, exp[:, :ncols].T.astype(np.int32)), mode


def _slice(r: D.BcReads, b0: int, b1: int, b: dict) -> D.BcReads:
    """A reference's slice of a device batch, as main.py's file-wide upload hands them out: the
    per-read pointers offset, n_reads shrunk, the whole batch's index fields left in place."""
    s = D.BcReads.from_buffer_copy(r)
    for f in ("pos", "cig_beg", "cig_n", "seq_nib"):
        setattr(s, f, getattr(r, f) + 4 * b0)
    s.n_reads = b1 - b0
    pos = b["pos"][b0:b1].astype(np.int64)
    span = np.array([sum(int(w) >> 4 for w in b["cigar"][cb: cb + cn] if int(w) & 15 in (0, 2, 3, 7, 8))
                     for cb, cn in zip(b["cig_beg"][b0:b1], b["cig_n"][b0:b1])], np.int64)
    s.max_span = int(span.max())
    s.max_end = int((pos + span).max())
    return s


@pytest.mark.parametrize("shape", ["rc", "tile_no_solo"])
def test_reads_index_on_device_slices(ctx, shape):
    """bc_reads_index builds a slice's index on the device (the CLI's per-reference slices of one
    upload); a slice that still carries the whole batch's index (index_tag mismatch)
    is counted from its own search / decode, never from the other batch's index."""
    ctx.set_shape(shape)
    rng = np.random.default_rng(61)
    L = 6_000
    b = random_batch(rng, L, 40_000)
    whole = D.DeviceReads(ctx, b)
    assert whole.r.index_tag != 0
    assert (whole.r.read_runs if shape == "rc" else whole.r.tile_reads)
    b0, b1 = 9_000, 31_000
    sb = dict(b, pos=b["pos"][b0:b1], cig_beg=b["cig_beg"][b0:b1], cig_n=b["cig_n"][b0:b1],
              seq_nib=b["seq_nib"][b0:b1])
    for mbq, k in ((0, 5), (20, 6)):
        exp, (br, _) = O.bcount(L, mbq, sb)
        assert br == -1
        got = []
        for mode in ("stale", "indexed"):
            s = _slice(whole.r, b0, b1, b)
            if mode == "indexed":
                nb = ctx.index_bytes(s, L)
                assert nb > 0
                mem = ctx.alloc(nb)
                ctx.index(s, L, mem.ptr, nb)
                assert s.index_tag != 0 and (s.read_runs if shape == "rc" else s.tile_reads)
            hist = ctx.alloc(4 * k * L)
            hist.zero()
            ctx.count(s, L, mbq, k, hist.ptr)
            assert ctx.range_error() == -1
            got.append(hist.download(np.int32, k * L).reshape(k, L))
        for g in got:
            assert np.array_equal(g, exp[:, :k].T.astype(np.int32))
    whole.free()


@pytest.mark.parametrize("seed,L,n,mbq,qual", [(71, 3_000, 20_000, 0, True), (72, 30_000, 60_000, 20, True),
                                               (73, 500, 5, 0, True), (74, 2_000_000, 3_000, 40, True),
                                               (75, 6_000, 40_000, 20, True), (76, 3_000, 60_000, 0, False),
                                               (77, 500, 3, 0, False)])
def test_device_sort_of_unsorted_batch(ctx, seed, L, n, mbq, qual):
    """bc_reads_sort: an unsorted batch put in start order on the device (bucketed sort of the
    starts + the sequence / quality copy into fixed slots); the sorted copy's starts are
    non-decreasing, it keeps every read, and every kernel shape on it gives the unsorted batch's
    counts (count.cpp's sums do not depend on the order)."""
    rng = np.random.default_rng(seed)
    b = random_batch(rng, L, n, sort=False)
    if not qual:
        b = dict(b, qual=None)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    r = D.DeviceReads(ctx, b)
    nb = ctx.sort_bytes(r)
    mem = ctx.alloc(nb)
    s = ctx.sort(r, mem.ptr, nb)
    assert s.sorted == 1 and s.n_reads == r.r.n_reads
    pos = np.zeros(s.n_reads, np.int32)
    D.check(D.lib().bc_memcpy_d2h(ctx.h, pos.ctypes.data, s.pos, pos.nbytes))
    ctx.sync()
    assert np.all(pos[1:] >= pos[:-1]) and np.array_equal(np.sort(b["pos"]), pos)
    for shape in ("auto", "tile_no_solo", "rc", "tile"):
        ctx.set_shape(shape)
        for k in (5, 6):
            nbi = ctx.index_bytes(s, L)
            imem = ctx.alloc(max(16, nbi))
            if nbi:
                ctx.index(s, L, imem.ptr, nbi)
            hist = ctx.alloc(4 * k * L)
            hist.zero()
            ctx.count(s, L, mbq, k, hist.ptr)
            assert ctx.range_error() == -1
            got = hist.download(np.int32, k * L).reshape(k, L)
            assert np.array_equal(got, exp[:, :k].T.astype(np.int32)), (shape, k)
    r.free()


@pytest.mark.parametrize("case", ["hot_start", "long_reference"])
def test_device_sort_bucket_extremes(ctx, case):
    """The bucketed sort's edges: 30,000 reads starting in 40 positions (one bucket holds far more
    records than a rank block keeps in registers: the overflow loops), and a reference of 2^24 +
    4,096 positions (too many starts for the buckets: the counting sort with global atomics).
    Sorted starts, and the sorted copy counts as the unsorted batch does."""
    rng = np.random.default_rng(93)
    if case == "hot_start":
        L, n = 5_000, 30_000
        b = random_batch(rng, L, n, sort=False, starts=lambda g, span: int(g.integers(200, 240)))
    else:
        L, n = (1 << 24) + 4_096, 2_000
        b = random_batch(rng, L, n, sort=False, starts=lambda g, span: int(g.integers(L - 3_000, L - span)))
    exp, (br, _) = O.bcount(L, 0, b)
    assert br == -1
    r = D.DeviceReads(ctx, b)
    nb = ctx.sort_bytes(r)
    mem = ctx.alloc(nb)
    s = ctx.sort(r, mem.ptr, nb)
    pos = np.zeros(s.n_reads, np.int32)
    D.check(D.lib().bc_memcpy_d2h(ctx.h, pos.ctypes.data, s.pos, pos.nbytes))
    ctx.sync()
    assert np.array_equal(np.sort(b["pos"]), pos)
    hist = ctx.alloc(4 * 5 * L)
    hist.zero()
    ctx.count(s, L, 0, 5, hist.ptr)
    assert ctx.range_error() == -1
    assert np.array_equal(hist.download(np.int32, 5 * L).reshape(5, L), exp[:, :5].T.astype(np.int32))
    hist.free()
    mem.free()
    r.free()


@pytest.mark.parametrize("mbq", [0, 30])
def test_device_sort_shrunk_slots_for_mixed_lengths(ctx, mbq):
    """A batch of short reads and one 6,000-base read: slots of the longest read's bytes would not
    fit the copy's buffer, so the device shrinks the slots (half the mean read) and the long read
    takes its bytes from the bump allocator past them -- decided on the device, no fallback, no
    host round trip; same counts, sorted starts, no error flag."""
    rng = np.random.default_rng(91)
    L, n = 20_000, 3_000
    pos = [int(x) for x in rng.integers(0, L - 60, n)]
    cigs = [[(0, 40)] for _ in range(n)]
    pos.append(100)
    cigs.append([(0, 3_000), (1, 3_000), (0, 10)])  # 6,010 query bases
    seqs = [synth.ACGT[rng.integers(0, 4, sum(ln for op, ln in c if op in (0, 1, 4, 7, 8)))] for c in cigs]
    quals = [rng.integers(0, 45, q.size).astype(np.uint8) for q in seqs]
    b = build_batch(pos, cigs, seqs, quals, sort=False)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    r = D.DeviceReads(ctx, b)
    nb = ctx.sort_bytes(r)
    mem = ctx.alloc(nb)
    s = ctx.sort(r, mem.ptr, nb)
    got_pos = np.zeros(s.n_reads, np.int32)
    D.check(D.lib().bc_memcpy_d2h(ctx.h, got_pos.ctypes.data, s.pos, got_pos.nbytes))
    ctx.sync()
    assert np.array_equal(got_pos, np.sort(b["pos"]))
    for shape in ("auto", "rc"):
        ctx.set_shape(shape)
        hist = ctx.alloc(4 * 5 * L)
        hist.zero()
        ctx.count(s, L, mbq, 5, hist.ptr)
        assert ctx.range_error() == -1
        assert np.array_equal(hist.download(np.int32, 5 * L).reshape(5, L), exp[:, :5].T.astype(np.int32)), shape
        hist.free()
    ctx.set_shape("auto")
    r.free()


def test_device_sort_read_longer_than_16_bits(ctx):
    """A read of 70,000 query bases (its length does not fit the bucketed record's 16 bits): the
    record keeps its source index and the copy re-reads its fields and CIGAR; counts exact."""
    rng = np.random.default_rng(94)
    L, n = 120_000, 2_000
    pos = [int(x) for x in rng.integers(0, L - 200, n)]
    cigs = [[(4, 3), (0, 150)] for _ in range(n)]
    pos.append(1_000)
    cigs.append([(0, 69_990), (2, 5), (0, 10)])
    seqs = [synth.ACGT[rng.integers(0, 4, sum(ln for op, ln in c if op in (0, 1, 4, 7, 8)))] for c in cigs]
    quals = [rng.integers(0, 45, q.size).astype(np.uint8) for q in seqs]
    b = build_batch(pos, cigs, seqs, quals, sort=False)
    exp, (br, _) = O.bcount(L, 0, b)
    assert br == -1
    r = D.DeviceReads(ctx, b)
    nb = ctx.sort_bytes(r)
    mem = ctx.alloc(nb)
    s = ctx.sort(r, mem.ptr, nb)
    hist = ctx.alloc(4 * 5 * L)
    hist.zero()
    ctx.count(s, L, 0, 5, hist.ptr)
    assert ctx.range_error() == -1
    assert np.array_equal(hist.download(np.int32, 5 * L).reshape(5, L), exp[:, :5].T.astype(np.int32))
    hist.free()
    mem.free()
    r.free()


def test_device_sort_flags_are_deferred(ctx):
    """bc_reads_sort only enqueues: a batch whose max_end is not truthful (a start past it) sorts
    without an error at the call, and bc_reads_sort_check then reports the bad start (BC_E_ARG);
    a truthful batch checks clean."""
    rng = np.random.default_rng(95)
    L, n = 4_000, 5_000
    b = random_batch(rng, L, n, sort=False)
    r = D.DeviceReads(ctx, b)
    nb = ctx.sort_bytes(r)
    mem = ctx.alloc(nb)
    ctx.sort(r, mem.ptr, nb, check_flags=False)
    ctx.sort_check(r, mem.ptr)  # clean
    bad = D.BcReads.from_buffer_copy(r.r)
    bad.max_end = 1_000  # starts beyond it exist
    nb2 = ctx.sort_bytes(bad)
    mem2 = ctx.alloc(nb2)
    s = ctx.sort(bad, mem2.ptr, nb2, check_flags=False)
    assert s.sorted == 1  # (no error at the call: the device has not run yet)
    with pytest.raises(D.BcError, match="outside"):
        ctx.sort_check(bad, mem2.ptr)
    for x in (mem, mem2):
        x.free()
    r.free()


def test_device_sort_in_a_graph(ctx):
    """The sort is capturable: sort + k_rc + kernel 2 of an unsorted C3-shaped batch replayed
    from one hipGraph twice give the oracle's counts."""
    rng = np.random.default_rng(96)
    L, n = 6_000, 120_000
    b = random_batch(rng, L, n, sort=False)
    exp, (br, _) = O.bcount(L, 0, b)
    assert br == -1
    r = D.DeviceReads(ctx, dict(b, qual=None))
    nb = ctx.sort_bytes(r)
    mem = ctx.alloc(nb)
    k = 5
    nf, nf2 = norm_factors(k)
    counts, cov, ent, sec = ctx.alloc(4 * k * L), ctx.alloc(4 * L), ctx.alloc(8 * L), ctx.alloc(8 * L)

    def step():
        s = ctx.sort(r, mem.ptr, nb, check_flags=False)
        ctx.pileup(s, L, 0, k, nf, nf2, counts.ptr, cov.ptr, None, ent.ptr, sec.ptr)

    step()  # (scratch allocated outside the capture)
    ctx.sync()
    g = ctx.capture(lambda: [step() for _ in range(2)])
    counts.zero()
    g.launch()
    ctx.sync()
    ctx.sort_check(r, mem.ptr)
    assert ctx.range_error() == -1
    assert np.array_equal(counts.download(np.int32, k * L).reshape(k, L), exp[:, :k].T.astype(np.int32))
    del g
    for x in (counts, cov, ent, sec, mem):
        x.free()
    r.free()


def scatter_sequences(b, rng):
    """The batch with every read's sequence bytes moved to a random place of a new buffer (its
    nibble parity and soft-clip offset kept): the same reads, no contiguous segment per chunk."""
    cig = b["cigar"]
    n = b["pos"].size
    q = np.zeros(n, np.int64)
    clip = np.zeros(n, np.int64)
    for i in range(n):
        ws = cig[b["cig_beg"][i]: b["cig_beg"][i] + b["cig_n"][i]]
        ops, lens = ws & 15, ws >> 4
        q[i] = int(lens[np.isin(ops, (0, 1, 4, 7, 8))].sum())
        clip[i] = int(lens[0]) if ops.size and ops[0] == 4 else 0
    start = (b["seq_nib"].astype(np.int64) - clip) // 2  # each read's first byte
    nbytes = (q + 1) // 2
    order = rng.permutation(n)
    off = np.zeros(n, np.int64)
    off[order] = np.concatenate([[0], np.cumsum(nbytes[order] + rng.integers(0, 3, n))[:-1]])
    seq = np.zeros(int((off + nbytes).max()) + 8, np.uint8)
    qual = np.zeros(2 * seq.size, np.uint8) if b.get("qual") is not None else None
    for i in range(n):
        seq[off[i]: off[i] + nbytes[i]] = b["seq"][start[i]: start[i] + nbytes[i]]
        if qual is not None:
            qual[2 * off[i]: 2 * (off[i] + nbytes[i])] = b["qual"][2 * start[i]: 2 * (start[i] + nbytes[i])]
    return dict(b, seq=seq, qual=qual, seq_nib=(2 * off + clip).astype(np.uint32))


@pytest.mark.parametrize("seed,L,n", [(81, 3_000, 40_000), (82, 30_000, 20_000), (83, 1_000, 300)])
@pytest.mark.parametrize("mbq", [0, 20])
def test_rc_gather_staging_of_scattered_sequence(ctx, seed, L, n, mbq):
    """A sorted batch whose reads' sequences lie scattered in their buffer (not one segment per
    chunk): k_rc copies each read's bytes into its own stage slot (gather staging; reads longer
    than a slot are walked from HBM) and counts exactly what the oracle counts."""
    rng = np.random.default_rng(seed)
    b = scatter_sequences(random_batch(rng, L, n), rng)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    r = D.DeviceReads(ctx, b)
    ctx.set_shape("rc")
    try:
        for k in (5, 6):
            hist = ctx.alloc(4 * k * L)
            hist.zero()
            ctx.count(r, L, mbq, k, hist.ptr)
            assert ctx.range_error() == -1
            got = hist.download(np.int32, k * L).reshape(k, L)
            assert np.array_equal(got, exp[:, :k].T.astype(np.int32)), k
            hist.free()
    finally:
        ctx.set_shape("auto")
        r.free()


def test_rc_event_image_range_error(ctx):
    """A read running past the reference end inside an imaged chunk: the reference's first
    offending read (std::out_of_range), nothing counted past L."""
    ctx.set_shape("rc")
    rng = np.random.default_rng(34)
    L = 5_000
    b = shaped_batch(rng, L + 400, 30_000, IMAGE_OK[:4])
    exp, (br, _) = O.bcount(L, 0, b)
    assert br != -1
    got, bad = gpu_count(ctx, b, L, 0, 5)
    assert bad == br


def test_kernel1_rpb_and_window_paths(ctx):
    """Same counts whatever the chunking: tiny chunks, huge chunks (global-atomic path), every
    waves-per-tile of the tiled kernel, with and without the sparse sweep."""
    rng = np.random.default_rng(9)
    b = random_batch(rng, 3_000, 8_000)
    exp, _ = O.bcount(3_000, 0, b)
    perm0 = np.random.default_rng(2).permutation(b["pos"].size)
    bu0 = dict(b, pos=b["pos"][perm0], cig_beg=b["cig_beg"][perm0], cig_n=b["cig_n"][perm0],
               seq_nib=b["seq_nib"][perm0])
    for rpb in (1, 7, 64, 4096, 30000):
        ctx.set_shape("auto", 0, rpb)
        got, bad = gpu_count(ctx, bu0, 3_000, 0, 6)
        assert bad == -1 and np.array_equal(got, exp.T.astype(np.int32)), rpb
    ctx.set_shape("auto")
    # unsorted order takes the event-parallel kernel: same counts
    perm = np.random.default_rng(1).permutation(b["pos"].size)
    bu = dict(b, pos=b["pos"][perm], cig_beg=b["cig_beg"][perm], cig_n=b["cig_n"][perm],
              seq_nib=b["seq_nib"][perm])
    got, bad = gpu_count(ctx, bu, 3_000, 0, 6)
    assert bad == -1 and np.array_equal(got, exp.T.astype(np.int32))
    for shape in ("tile", "tile_no_solo"):
        for waves in (1, 2, 4, 8):
            ctx.set_shape(shape, waves)
            got, bad = gpu_count(ctx, b, 3_000, 0, 6)
            assert bad == -1 and np.array_equal(got, exp.T.astype(np.int32)), (shape, waves)
    for bad_waves in (3, 5, 6, 7, 16):  # must divide the block's waves
        with pytest.raises(D.BcError):
            ctx.set_shape("tile", bad_waves)


def test_kernel1_range_error_first_read(ctx):
    rng = np.random.default_rng(4)
    b = random_batch(rng, 1_000, 500)
    L = 1_000
    # shrink the reference so that some reads run past its end
    L2 = int(np.percentile(b["pos"], 80))
    exp, (br, bp) = O.bcount(L2, 0, b)
    assert br >= 0
    _, bad = gpu_count(ctx, b, L2, 0, 6)
    assert bad == br
    # high quality threshold: only counted events can trip the check
    exp40, (br40, _) = O.bcount(L2, 40, b)
    _, bad40 = gpu_count(ctx, b, L2, 40, 6)
    assert bad40 == br40


def gpu_pileup(ctx, b, L, mbq, k):
    r = D.DeviceReads(ctx, b)
    assert r.r.sorted == 1
    bufs = [ctx.alloc(max(8, n)) for n in (4 * k * L, 4 * L, 8 * k * L, 8 * L, 8 * L)]
    nf, nf2 = norm_factors(k)
    ctx.pileup(r, L, mbq, k, nf, nf2, *[x.ptr for x in bufs])
    bad = ctx.range_error()
    out = (bufs[0].download(np.int32, k * L).reshape(k, L), bufs[1].download(np.int32, L),
           bufs[2].download(np.float64, k * L).reshape(k, L), bufs[3].download(np.float64, L),
           bufs[4].download(np.float64, L))
    return out, bad


@pytest.mark.parametrize("seed,L,n", [(11, 700, 900), (12, 29_903, 30_000), (13, 5_000, 60_000),
                                      (14, 2_000_000, 3_000), (15, 64, 50), (16, 65, 80)])
@pytest.mark.parametrize("mbq,show_n", [(0, False), (20, True), (40, False)])
@pytest.mark.parametrize("path", ["tile", "rc"])
def test_fused_pileup_matches_oracle(ctx, seed, L, n, mbq, show_n, path):
    ctx.set_shape(path)
    rng = np.random.default_rng(seed)
    b = random_batch(rng, L, n)
    k = 6 if show_n else 5
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    (cnt, cov, pc, ent, sec), bad = gpu_pileup(ctx, b, L, mbq, k)
    assert bad == -1
    ocov, opc, oent, osec = O.stats(exp, show_n)
    assert np.array_equal(cnt, exp[:, :k].T.astype(np.int32))
    assert np.array_equal(cov, ocov) and np.array_equal(pc, opc)
    assert np.max(np.abs(ent - oent)) <= 1e-6 and np.max(np.abs(sec - osec)) <= 1e-6
    assert np.array_equal(ent, oent) and np.array_equal(sec, osec)  # glibc log2 on the device


def _tile_index(ctx, r):
    n = int(r.r.n_tiles)
    if n == 0 or not r.r.tile_reads:
        return None
    out = np.zeros(2 * n, np.int32)
    D.check(D.lib().bc_memcpy_d2h(ctx.h, out.ctypes.data, r.r.tile_reads, out.nbytes))
    ctx.sync()
    return out.reshape(n, 2)


@pytest.mark.parametrize("seed,L,n", [(21, 29_903, 30_000), (22, 700, 5_000), (23, 1_000_000, 2_000)])
def test_tile_index_matches_searchsorted(ctx, seed, L, n):
    """bc_reads_upload's tile index (bc_reads.tile_reads) is the range the tiled kernel would
    search for: [first pos > 64t - max_span, first pos >= 64t + 64) for every tile up to
    max_end; absent for sparse batches (more tiles than reads / 16)."""
    rng = np.random.default_rng(seed)
    b = random_batch(rng, L, n)
    r = D.DeviceReads(ctx, b)
    idx = _tile_index(ctx, r)
    tiles = (int(r.r.max_end) + 63) // 64
    if tiles > len(b["pos"]) // 16:
        assert idx is None
    else:
        t = np.arange(tiles, dtype=np.int64) * 64
        pos = b["pos"].astype(np.int64)
        assert idx.shape == (tiles, 2)
        assert np.array_equal(idx[:, 0], np.searchsorted(pos, t - int(r.r.max_span) + 1, "left"))
        assert np.array_equal(idx[:, 1], np.searchsorted(pos, t + 64, "left"))
    r.free()


@pytest.mark.parametrize("L_extra", [0, 5_000, -120])
def test_pileup_same_without_tile_index(ctx, L_extra):
    """The tiled kernel gives identical outputs (and the same first out-of-range read) from the
    tile index and from its own search, including tiles past the index (L > max_end) and edge
    tiles past L (reads beyond the reference end)."""
    ctx.set_shape("tile_no_solo")
    rng = np.random.default_rng(31)
    L0 = 8_000
    b = random_batch(rng, L0, 12_000)
    L = L0 + L_extra
    outs = []
    for use in (True, False):
        r = D.DeviceReads(ctx, b)
        assert (r.r.n_tiles > 0) and r.r.tile_reads
        if not use:
            r.r.tile_reads = None
            r.r.n_tiles = 0
        k = 5
        bufs = [ctx.alloc(max(8, x)) for x in (4 * k * L, 4 * L, 8 * k * L, 8 * L, 8 * L)]
        nf, nf2 = norm_factors(k)
        try:
            ctx.pileup(r, L, 0, k, nf, nf2, *[x.ptr for x in bufs])
            err = None
        except D.BcError as e:
            err = e.code
        bad = ctx.range_error()
        outs.append((err, bad, bufs[0].download(np.int32, k * L), bufs[1].download(np.int32, L),
                     bufs[3].download(np.float64, L)))
        r.free()
    (e1, b1, *o1), (e2, b2, *o2) = outs
    assert e1 == e2 and b1 == b2
    exp, (br, _) = O.bcount(L, 0, b)
    assert b1 == br and (br >= 0) == (L_extra < 0)  # reads beyond a shortened reference
    if br == -1:
        assert np.array_equal(o1[0].reshape(5, L), exp[:, :5].T.astype(np.int32))
    for x, y in zip(o1, o2):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("path", ["tile", "rc"])
def test_fused_pileup_range_error(ctx, path):
    ctx.set_shape(path)
    rng = np.random.default_rng(21)
    b = random_batch(rng, 2_000, 3_000)
    for L2 in (1_990, 1_900, 1_000, 64):
        for mbq in (0, 30):
            _, (br, _) = O.bcount(L2, mbq, b)
            _, bad = gpu_pileup(ctx, b, L2, mbq, 5)
            assert bad == br, (L2, mbq)


@pytest.mark.parametrize("show_n", [False, True])
def test_kernel2_matches_oracle(ctx, show_n):
    rng = np.random.default_rng(7)
    L = 200_000
    c = rng.integers(0, 50, (L, 6)).astype(np.uint32)
    c[rng.random((L, 6)) < 0.5] = 0
    c[:1000] = 0
    c[1000:2000, 1:] = 0                      # single nonzero column (cov2 == 0)
    c[2000:3000] = 7                          # ties (first argmax)
    c[3000:4000] = rng.integers(0, 3_000_000, (1000, 6))  # deep coverage
    k = 6 if show_n else 5
    cov, pc, ent, sec = O.stats(c, show_n)
    planes = np.ascontiguousarray(c[:, :k].T.astype(np.int32))
    hist = ctx.alloc(planes.nbytes).upload(planes)
    dcov, dpc, dent, dsec = (ctx.alloc(4 * L), ctx.alloc(8 * k * L), ctx.alloc(8 * L),
                             ctx.alloc(8 * L))
    nf, nf2 = norm_factors(k)
    ctx.stats(hist.ptr, L, k, nf, nf2, dcov.ptr, dpc.ptr, dent.ptr, dsec.ptr)
    gcov = dcov.download(np.int32, L)
    gpc = dpc.download(np.float64, k * L).reshape(k, L)
    gent, gsec = dent.download(np.float64, L), dsec.download(np.float64, L)
    assert np.array_equal(gcov, cov)
    assert np.array_equal(gpc, pc)              # IEEE division and multiply: exact
    tol = 1e-6                                  # north_star entropy tolerance
    assert np.max(np.abs(gent - ent)) <= tol and np.max(np.abs(gsec - sec)) <= tol
    exact = float(np.mean(gent == ent)), float(np.mean(gsec == sec))
    print(f"entropy bit-exact fraction: {exact[0]:.6f}, secondary: {exact[1]:.6f}")
    # kernel 2 evaluates glibc's log2 algorithm (bc_log2.h): bit-identical to math.log2
    assert exact == (1.0, 1.0)
    # printed values (3 dp) must agree
    for a, e in ((gent, ent), (gsec, sec)):
        assert [str(round(x, 3)) for x in a[:20000].tolist()] == [
            str(round(x, 3)) for x in e[:20000].tolist()]


@pytest.mark.parametrize("L", [1, 7, 8, 9, 127, 128, 129, 136, 1000, 8191, 8192, 8193, 29_903,
                               100_000, 1_000_003, 2_203_000, 6_000_001])
def test_summary_matches_numpy(ctx, L):
    rng = np.random.default_rng(L)
    cov = rng.integers(0, 5000, L).astype(np.int32)
    cov[rng.random(L) < 0.2] = 0
    ent = rng.random(L)
    ent[cov == 0] = 1.0
    dc, de = ctx.alloc(4 * L).upload(cov), ctx.alloc(8 * L).upload(ent)
    work = ctx.alloc(D.summary_work_bytes(L))
    out = ctx.alloc(32)
    ctx.summary(dc.ptr, de.ptr, L, work.ptr, out.ptr)
    s = out.download(np.float64, 4)
    assert s[0] == np.mean(cov.tolist())
    assert s[1] == np.mean(ent.tolist())
    assert int(s[2]) == int(np.count_nonzero(cov))


@pytest.mark.parametrize("wmax,ties", [(9000, False), (600, True)])
def test_amplicons_match_numpy(ctx, wmax, ties):
    """k_amplicon against numpy's mean / median per window (main.py:519-551): wide windows (the
    radix-select medians) and amplicon-sized ones (<= 512 positions: one wave's bitonic sort per
    array), with many tied values, odd and even lengths, empty and clipped windows."""
    rng = np.random.default_rng(3 + wmax)
    L = 30_000
    cov = rng.integers(0, 6 if ties else 3000, L).astype(np.int32)
    ent = rng.integers(0, 4, L) / 3.0 if ties else rng.random(L)
    sec = rng.random(L)
    if ties:
        sec[rng.random(L) < 0.5] = 1.0
    ent[:500] = 1.0
    tiles = [(int(a), int(a + w)) for a, w in zip(rng.integers(-50, L, 200), rng.integers(-5, wmax, 200))]
    tiles += [(0, 0), (L - 1, L + 10), (5, 4), (L + 5, L + 9), (0, L - 1)]
    lo = np.array([t[0] for t in tiles], np.int64)
    hi = np.array([t[1] for t in tiles], np.int64)
    dc, de, ds = ctx.alloc(4 * L).upload(cov), ctx.alloc(8 * L).upload(ent), ctx.alloc(8 * L).upload(sec)
    dlo, dhi, dout = ctx.alloc(lo.nbytes).upload(lo), ctx.alloc(hi.nbytes).upload(hi), ctx.alloc(48 * len(tiles))
    ctx.amplicons(dc.ptr, de.ptr, ds.ptr, L, dlo.ptr, dhi.ptr, len(tiles), dout.ptr)
    got = dout.download(np.float64, 6 * len(tiles)).reshape(-1, 6)
    exp = O.amplicons(cov, ent, sec, tiles)
    for i, e in enumerate(exp):
        assert got[i].tolist() == [float(x) for x in e], (i, tiles[i])


@pytest.mark.parametrize("L,n,mbq,k", [(8192 * 3 + 1711, 60_000, 0, 5), (8192 * 2, 40_000, 20, 6),
                                        (5_000, 30_000, 0, 5), (40_003, 50_000, 0, 6),
                                        # the partial buffer's tree: below numpy's 8-element rule,
                                        # one split past a 128-leaf, a reference shorter than a leaf
                                        (8192 + 5, 20_000, 0, 5), (8192 + 130, 20_000, 0, 6), (100, 2_000, 0, 5)])
def test_pileup_summary_amplicons_fused_tail(ctx, L, n, mbq, k):
    """bc_pileup_summary_amplicons on the read-chunked path (kernel 1, kernel 2 with numpy's leaf
    partials, then ONE launch for the summary fold and every window): the summary's four numbers
    equal numpy over the oracle's coverage / entropies (main.py:469-499), every window's means and
    medians the oracle's (main.py:519-551) -- amplicon-sized windows (rank-counted medians), wide
    ones (radix select), empty and clipped ones -- and bc_pileup_summary (no windows, summary only
    too) gives the same summary."""
    rng = np.random.default_rng(L + n)
    b = random_batch(rng, L, n)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    ocov, _, oent, osec = O.stats(exp, k == 6)
    want = [np.mean(ocov.astype(np.int64)), np.mean(oent), float(np.count_nonzero(ocov)), float(ocov.astype(np.int64).sum())]
    tiles = [(int(a), int(a + w)) for a, w in zip(rng.integers(-20, L, 60), rng.integers(-3, 420, 60))]
    tiles += [(0, 0), (L - 1, L + 10), (5, 4), (100, 100 + 1_500), (0, L - 1)]
    # every count of sorted 64-key runs (n = 64, 65, 449, 512), the first radix-select size (513),
    # and enough windows for more blocks than CUs (3 per window + the summary's)
    tiles += [(7, 7 + 63), (7, 7 + 64), (3, 3 + 448), (11, 11 + 511), (2, 2 + 512)]
    tiles += [(int(a), int(a + w)) for a, w in zip(rng.integers(0, L, 30), rng.integers(200, 280, 30))]
    lo = np.array([t[0] for t in tiles], np.int64)
    hi = np.array([t[1] for t in tiles], np.int64)
    ctx.set_shape("rc")
    try:
        nf, nf2 = norm_factors(k)
        r = D.DeviceReads(ctx, b)
        counts, cov, ent, sec = ctx.alloc(4 * k * L), ctx.alloc(4 * L), ctx.alloc(8 * L), ctx.alloc(8 * L)
        work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        dlo, dhi, damp = ctx.alloc(lo.nbytes).upload(lo), ctx.alloc(hi.nbytes).upload(hi), ctx.alloc(48 * len(tiles))
        for _ in range(2):  # (the second call on the scratch the first left zeroed)
            ctx.pileup_summary_amplicons(r, L, mbq, k, nf, nf2, counts.ptr, cov.ptr, ent.ptr, sec.ptr, work.ptr,
                                         dout.ptr, dlo.ptr, dhi.ptr, len(tiles), damp.ptr)
            assert ctx.range_error() == -1
            assert dout.download(np.float64, 4).tolist() == want
            got = damp.download(np.float64, 6 * len(tiles)).reshape(-1, 6)
            for i, e in enumerate(O.amplicons(ocov, oent, osec, tiles)):
                assert got[i].tolist() == [float(x) for x in e], (i, tiles[i])
        assert np.array_equal(counts.download(np.int32, k * L).reshape(k, L), exp[:, :k].T.astype(np.int32))
        for outs in ((counts.ptr, cov.ptr, ent.ptr, sec.ptr), (None, None, None, None)):
            dout.zero()
            ctx.pileup_summary(r, L, mbq, k, nf, nf2, outs[0], outs[1], None, outs[2], outs[3], work.ptr, dout.ptr)
            assert dout.download(np.float64, 4).tolist() == want
        r.free()
    finally:
        ctx.set_shape("auto")


# ------------------------------------------------------------------ CLI vs reference goldens
def _run_cli(argv):
    from basecount_amd.main import run

    buf = io.BytesIO()
    txt = io.TextIOWrapper(buf, encoding="utf-8", write_through=True)
    with contextlib.redirect_stdout(txt):
        run(argv)
        txt.flush()
    return buf.getvalue()


# Streamed in batches far smaller than the file (main.batch_records): every reference of the
# edge / error BAMs (<= 116 records, 4 references) crosses batch boundaries, faults land in
# later batches, and c1 / mixed are counted by accumulation over 4-14 batches.
def _stream_batches(bam: str) -> str:
    return "3" if bam.startswith(("edge", "err")) else "300"


@pytest.mark.parametrize("stream", [False, True])
def test_cli_matches_reference_goldens(golden, manifest, monkeypatch, stream):
    n = 0
    cwd = os.getcwd()
    os.chdir(golden)
    try:
        for name, c in sorted(manifest.items()):
            if c.get("hashseed", "0") != "0" or name.startswith("err_order"):
                continue  # set-order dependent: test_cli_hashseed_cases_byte_exact
            if stream:
                monkeypatch.setenv("BASECOUNT_BATCH_RECORDS", _stream_batches(c["bam"]))
            argv = [c["bam"]] + c["args"]
            summ = "--summarise" in c["args"] or "--summarise-with-bed" in c["args"]
            if c["returncode"] != 0:
                with pytest.raises(BaseException) as ei:
                    _run_cli(argv)
                exc = ei.value
                line = f"{type(exc).__name__}: {exc}".splitlines()[0]
                if isinstance(exc, KeyError):
                    line = f"KeyError: {exc}"
                assert line == c["error"], name
                n += 1
                continue
            with open(c["stdout"], "rb") as fh:
                exp = gzip.decompress(fh.read()).decode()
            got = _run_cli(argv).decode()
            h1, b1 = O.split_blocks(got, summ)
            h2, b2 = O.split_blocks(exp, summ)
            assert h1 == h2 and b1 == b2, name
            if len(b2) == 1:
                assert got == exp, name
            n += 1
    finally:
        os.chdir(cwd)
    assert n >= 40


@pytest.mark.parametrize("stream", [False, True])
def test_cli_hashseed_cases_byte_exact(golden, manifest, stream):
    """Multi-reference output order and first-error choice follow the set order (main.py:92)."""
    env0 = dict(os.environ, PYTHONPATH=REPO)
    for name, c in sorted(manifest.items()):
        if c.get("hashseed", "0") == "0" and not name.startswith(("edge_q0_m0", "err_order")):
            continue
        env = dict(env0, PYTHONHASHSEED=c.get("hashseed", "0"))
        if stream:
            env["BASECOUNT_BATCH_RECORDS"] = _stream_batches(c["bam"])
        p = subprocess.run([sys.executable, "-m", "basecount_amd", c["bam"]] + c["args"],
                           cwd=golden, env=env, capture_output=True, timeout=300)
        if c["returncode"] != 0:
            assert p.returncode != 0, name
            assert c["error"] in p.stderr.decode(), name
        else:
            with open(os.path.join(golden, c["stdout"]), "rb") as fh:
                assert p.stdout == gzip.decompress(fh.read()), name


def test_bcount_adapter_matches_reference_vectors(golden):
    import json

    from basecount_amd.count import bcount

    with open(os.path.join(golden, "bcount", "vectors.json")) as fh:
        vec = json.load(fh)
    for name, v in vec.items():
        ct = [[tuple(t) for t in c] for c in v["ctuples"]]
        if "error" in v:
            with pytest.raises(IndexError) as ei:
                bcount(v["ref_len"], v["mbq"], v["reads"], v["qualities"], v["starts"], ct)
            assert str(ei.value) == v["error"][1]
        else:
            assert bcount(v["ref_len"], v["mbq"], v["reads"], v["qualities"], v["starts"], ct) \
                == v["expected"], name
    with pytest.raises(TypeError):
        bcount(10, -1, [], [], [], [])
    with pytest.raises(TypeError):
        bcount(10, 0, ["A"], [None], [0], [[(0, 1)]])


# ------------------------------------------------------------------ full-size configurations
@pytest.mark.parametrize("cfg,mmq,mbq", [("c2", 0, 0), ("c3", 0, 0), ("c3", 30, 20)])
@pytest.mark.parametrize("path", ["tile", "rc"])
def test_full_size_configs_exact(ctx, cfg, mmq, mbq, path):
    ctx.set_shape(path)
    rs = synth.make_config(cfg)
    b = synth.batch_arrays(rs, 0, mmq)
    L = rs.lengths[0]
    exp, (br, _) = O.bcount(L, mbq, b)
    got, bad = gpu_count(ctx, b, L, mbq, 5)
    assert br == -1 and bad == -1
    assert np.array_equal(got, exp[:, :5].T.astype(np.int32))
    if mbq == 0 and mmq == 0:  # every ref-consuming event is counted: checksum of checksums
        assert int(got.sum()) + int(exp[:, 5].sum()) == synth.ref_events(rs)


@pytest.mark.parametrize("cfg,path", [("c3", "auto"), ("c3", "tile"), ("c3", "rc"), ("c2", "auto")])
def test_full_size_fused_pileup(ctx, cfg, path):
    """The bench's step (bc_pileup) on the full C3 batch, and on the full C2 batch (the
    headline's fused k_pileup with statistics): counts, coverage and
    percentages exact, entropies bit-identical (and within north_star's 1e-6)."""
    ctx.set_shape(path)
    rs = synth.make_config(cfg)
    b = synth.batch_arrays(rs, 0, 0)
    L = rs.lengths[0]
    exp, (br, _) = O.bcount(L, 0, b)
    (cnt, cov, pc, ent, sec), bad = gpu_pileup(ctx, b, L, 0, 5)
    assert br == -1 and bad == -1
    assert np.array_equal(cnt, exp[:, :5].T.astype(np.int32))
    ocov, opc, oent, osec = O.stats(exp, False)
    assert np.array_equal(cov, ocov) and np.array_equal(pc, opc)
    assert np.max(np.abs(ent - oent)) <= 1e-6 and np.max(np.abs(sec - osec)) <= 1e-6
    assert np.array_equal(ent, oent) and np.array_equal(sec, osec)


@pytest.mark.parametrize("mbq,ncols", [(0, 5), (20, 6)])
def test_rc_64bit_indices_chromosome_scale(ctx, mbq, ncols):
    """k_rc's int64_t instantiation (taken when L or n >= 2^27, i.e. deep
    batches on human chr1-chr12 / X) against the oracle: L = 2^27 + 10,000, 20,000 mixed-CIGAR
    reads near the far end and a few at 0, shape forced to rc; then the same batch with the
    reference cut short, whose first offending read must be the oracle's (count.cpp:17,60-65)."""
    ctx.set_shape("rc")
    L = (1 << 27) + 10_000
    rng = np.random.default_rng(77 + mbq)
    b = shaped_batch(rng, 20_000, 20_000, IMAGE_DEEP + FALLBACK)
    far = np.arange(b["pos"].size) >= 40  # the 40 leftmost reads stay near position 0
    b["pos"] = (b["pos"].astype(np.int64) + np.where(far, L - 20_000, 0)).astype(np.int32)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    got, bad = gpu_count(ctx, b, L, mbq, ncols)
    assert bad == -1
    exp = exp[:, :ncols]
    assert int(got.sum(dtype=np.int64)) == int(exp.sum(dtype=np.int64))
    for lo, hi in ((0, 20_000), (L - 20_000, L)):
        assert np.array_equal(got[:, lo:hi], exp[lo:hi].T.astype(np.int32)), (lo, hi)
    del got, exp
    L2 = L - 60  # reads now run past the end: std::out_of_range in the reference
    _, (br2, _) = O.bcount(L2, mbq, b)
    assert br2 >= 0
    _, bad2 = gpu_count(ctx, b, L2, mbq, ncols)
    assert bad2 == br2


@pytest.mark.parametrize("mbq,k", [(0, 5), (20, 6)])
def test_rc_pileup_64bit_chromosome_scale(ctx, mbq, k):
    """the pileup chain at chromosome scale (int64_t k_rc + k_stats_lane,
    L = 2^27 + 10,000) against the oracle on both 20,000-position windows: counts, coverage,
    percentages and both entropies (bit-identical; the 1e-6 bound asserted too)."""
    ctx.set_shape("rc")
    L = (1 << 27) + 10_000
    rng = np.random.default_rng(91 + mbq)
    b = shaped_batch(rng, 20_000, 20_000, IMAGE_DEEP + FALLBACK)
    far = np.arange(b["pos"].size) >= 40
    b["pos"] = (b["pos"].astype(np.int64) + np.where(far, L - 20_000, 0)).astype(np.int32)
    exp, (br, _) = O.bcount(L, mbq, b)
    assert br == -1
    nf, nf2 = norm_factors(k)
    r = D.DeviceReads(ctx, b)
    bufs = [ctx.alloc(x) for x in (4 * k * L, 4 * L, 8 * k * L, 8 * L, 8 * L)]
    ctx.pileup(r, L, mbq, k, nf, nf2, *(x.ptr for x in bufs))
    assert ctx.range_error() == -1
    for lo, hi in ((0, 20_000), (L - 20_000, L)):
        n = hi - lo
        cov_o, pc_o, ent_o, sec_o = O.stats(exp[lo:hi], k == 6)
        for c in range(k):
            got = bufs[0].download(np.int32, n, offset_bytes=4 * (c * L + lo))
            assert np.array_equal(got, exp[lo:hi, c].astype(np.int32)), (lo, c)
            gpc = bufs[2].download(np.float64, n, offset_bytes=8 * (c * L + lo))
            assert np.array_equal(gpc, pc_o[c]), (lo, c)
        assert np.array_equal(bufs[1].download(np.int32, n, offset_bytes=4 * lo), cov_o)
        ent, sec = bufs[3].download(np.float64, n, offset_bytes=8 * lo), bufs[4].download(np.float64, n, offset_bytes=8 * lo)
        assert np.max(np.abs(ent - ent_o)) <= 1e-6 and np.max(np.abs(sec - sec_o)) <= 1e-6
        assert np.array_equal(ent, ent_o) and np.array_equal(sec, sec_o)
    for x in bufs:
        x.free()
    r.free()


@pytest.mark.parametrize("L,n,mbq,show_n", [
    (8192 * 9, 3_000, 0, False),          # whole buffers only
    (8192 * 9 + 517, 3_000, 20, True),    # a partial last buffer (computed by the tail kernel)
    (8191, 400, 0, False),                # no whole buffer
    (200_000, 20, 0, False),              # read-free buffers
    (1_000_003, 5_000, 30, False),
    (29_903, 60_000, 0, False),           # deep enough for the tiled kernel: plain pileup + summary
])
def test_pileup_summary_matches_separate_calls(ctx, L, n, mbq, show_n):
    """bc_pileup_summary (numpy's buffer partials computed inside the sparse sweep) gives the
    same per-position outputs and the same summary doubles, bit for bit, as bc_pileup followed
    by bc_summary, and the summary equals numpy's mean over the arrays (main.py:469-499)."""
    rng = np.random.default_rng(L + n)
    b = random_batch(rng, L, n)
    k = 6 if show_n else 5
    nf, nf2 = norm_factors(k)
    r = D.DeviceReads(ctx, b)
    outs = []
    for fused in (False, True):
        bufs = [ctx.alloc(max(8, x)) for x in (4 * k * L, 4 * L, 8 * L, 8 * L)]
        work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        work.zero()
        if fused:
            ctx.pileup_summary(r, L, mbq, k, nf, nf2, bufs[0].ptr, bufs[1].ptr, None, bufs[2].ptr,
                               bufs[3].ptr, work.ptr, dout.ptr)
        else:
            ctx.pileup(r, L, mbq, k, nf, nf2, bufs[0].ptr, bufs[1].ptr, None, bufs[2].ptr, bufs[3].ptr)
            ctx.summary(bufs[1].ptr, bufs[2].ptr, L, work.ptr, dout.ptr)
        assert ctx.range_error() == -1
        outs.append((bufs[0].download(np.int32, k * L), bufs[1].download(np.int32, L),
                     bufs[2].download(np.float64, L), bufs[3].download(np.float64, L),
                     dout.download(np.float64, 4)))
    for a, b2 in zip(*outs):
        assert np.array_equal(a, b2)
    cov, ent, s = outs[1][1], outs[1][2], outs[1][4]
    assert s[0] == np.mean(cov.astype(np.int64)) and s[1] == np.mean(ent)
    assert int(s[2]) == int(np.count_nonzero(cov)) and int(s[3]) == int(cov.astype(np.int64).sum())
    # summary only: no per-position outputs at all, the same four doubles
    work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
    for rep in range(2):  # (the second call reuses the context's tail scratch)
        work.zero()
        ctx.pileup_summary(r, L, mbq, k, nf, nf2, None, None, None, None, None, work.ptr, dout.ptr)
        assert ctx.range_error() == -1
        assert np.array_equal(dout.download(np.float64, 4), s), rep


@pytest.mark.parametrize("L,n,mbq,show_n,layout", [
    (8192 * 64, 6_000, 0, False, "uniform"),
    (8192 * 64 + 4_321, 6_000, 20, True, "uniform"),
    (8192 * 200 + 17, 20_000, 0, False, "clusters"),     # hot spots: many leaves two reads share
    (8192 * 200 + 17, 20_000, 30, True, "clusters"),
    (8192 * 30, 3_000, 0, False, "boundaries"),          # reads across leaf / quarter / buffer edges
    (3_000_000, 1_500, 0, False, "uniform"),
])
def test_summary_only_read_parallel(ctx, L, n, mbq, show_n, layout):
    """The summary-only path of a sparse batch (bc_sum.hip: counted positions per 128-position
    leaf, exact walks of the leaves two reads share, each 8192-position buffer's 64 leaves added
    in numpy's tree order into whole-buffer partials) gives exactly the
    four numbers numpy computes over the oracle's coverage and entropies (main.py:469-499), with
    mixed CIGARs, quality thresholds, N columns, dense clusters and partial last buffers; and
    again on the same context (its leaf scratch is left zeroed)."""
    rng = np.random.default_rng(L + n + mbq)
    if layout == "clusters":
        centers = rng.integers(0, L - 400, 60)
        starts = lambda g, span: int(min(L - span - 1, centers[g.integers(0, 60)] + g.integers(0, 300)))
    elif layout == "boundaries":
        starts = lambda g, span: int(max(0, min(L - span - 1, 128 * g.integers(1, L // 128) - g.integers(0, 40))))
    else:
        starts = None
    b = random_batch(rng, L, n, starts=starts)
    k = 6 if show_n else 5
    nf, nf2 = norm_factors(k)
    exp, (bad, _) = O.bcount(L, mbq, b)
    assert bad == -1
    cov, _, ent, _ = O.stats(exp, show_n)
    want = np.array([np.mean(cov.astype(np.int64)), np.mean(ent), np.count_nonzero(cov),
                     cov.astype(np.int64).sum()], np.float64)
    r = D.DeviceReads(ctx, b)
    work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
    for rep in range(2):
        work.zero()
        ctx.pileup_summary(r, L, mbq, k, nf, nf2, None, None, None, None, None, work.ptr, dout.ptr)
        assert ctx.range_error() == -1
        assert np.array_equal(dout.download(np.float64, 4), want), (rep, dout.download(np.float64, 4), want)


def test_summary_only_scratch_reuse_across_lengths():
    """One context, references of decreasing then increasing length with many shared leaves:
    the leaf scratch (grown once, laid out by its capacity) must be all zero again for each call
    whatever the previous call's length (a length-dependent layout once read stale slots)."""
    c = D.Context(0)
    k = 5
    nf, nf2 = norm_factors(k)
    for i, L in enumerate((8192 * 300, 8192 * 12, 8192 * 40 + 3_000, 8192 * 5 + 1, 8192 * 150 + 77)):
        rng = np.random.default_rng(1234 + i)
        centers = rng.integers(0, L - 400, 25)
        starts = lambda g, span: int(min(L - span - 1, centers[g.integers(0, 25)] + g.integers(0, 250)))
        b = random_batch(rng, L, 4_000 if L > 100_000 else 600, starts=starts)
        exp, (bad, _) = O.bcount(L, 0, b)
        cov, _, ent, _ = O.stats(exp, False)
        want = np.array([np.mean(cov.astype(np.int64)), np.mean(ent), np.count_nonzero(cov),
                         cov.astype(np.int64).sum()], np.float64)
        r = D.DeviceReads(c, b)
        work, dout = c.alloc(D.summary_work_bytes(L)), c.alloc(32)
        work.zero()
        c.pileup_summary(r, L, 0, k, nf, nf2, None, None, None, None, None, work.ptr, dout.ptr)
        assert c.range_error() == -1
        assert np.array_equal(dout.download(np.float64, 4), want), (L, dout.download(np.float64, 4), want)
        r.free()
    c.close()


@pytest.mark.parametrize("mbq", [0, 20])
def test_summary_only_read_parallel_range_error(ctx, mbq):
    """Reads running past the reference end in the summary-only path: the first offending read
    is the oracle's (count.cpp:60-65,85, std::out_of_range)."""
    rng = np.random.default_rng(99 + mbq)
    L0 = 8192 * 12 + 300
    b = random_batch(rng, L0, 2_000)
    w, ob = b["cigar"], b["cig_beg"].astype(np.int64)
    span = np.array([sum(int(x) >> 4 for x in w[ob[i]: ob[i] + int(b["cig_n"][i])] if int(x) & 15 in (0, 2, 3, 7, 8))
                     for i in range(b["pos"].size)])
    e = int((b["pos"].astype(np.int64) + span).max())
    for L in (e - 20, e - 60, 8192 * 12):
        _, (bad, _) = O.bcount(L, mbq, b)
        assert bad >= 0
        r = D.DeviceReads(ctx, b)
        work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        ctx.pileup_summary(r, L, mbq, 5, *norm_factors(5), None, None, None, None, None, work.ptr, dout.ptr)
        assert ctx.range_error() == bad, L
        r.free()


@pytest.mark.parametrize("L,n", [(8192 * 40 + 3_000, 30), (8192 * 3, 0), (5_000_000, 200)])
def test_pileup_summary_only_sparse_edges(ctx, L, n):
    """The summary-only sweep on read-free quarters (one constant store each), a batch with no
    reads, and a reference whose last buffer is partial: the summary equals numpy's over the
    storing call's arrays."""
    rng = np.random.default_rng(L + 7)
    b = random_batch(rng, L, n) if n else random_batch(rng, L, 1)
    if not n:
        b = dict(b, pos=b["pos"][:0], cig_beg=b["cig_beg"][:0], cig_n=b["cig_n"][:0], seq_nib=b["seq_nib"][:0])
    k = 5
    nf, nf2 = norm_factors(k)
    r = D.DeviceReads(ctx, b)
    bufs = [ctx.alloc(max(8, x)) for x in (4 * k * L, 4 * L, 8 * L, 8 * L)]
    work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
    ctx.pileup_summary(r, L, 0, k, nf, nf2, bufs[0].ptr, bufs[1].ptr, None, bufs[2].ptr, bufs[3].ptr,
                       work.ptr, dout.ptr)
    want = dout.download(np.float64, 4)
    cov, ent = bufs[1].download(np.int32, L), bufs[2].download(np.float64, L)
    assert want[0] == np.mean(cov.astype(np.int64)) and want[1] == np.mean(ent)
    work.zero()
    ctx.pileup_summary(r, L, 0, k, nf, nf2, None, None, None, None, None, work.ptr, dout.ptr)
    assert ctx.range_error() == -1
    assert np.array_equal(dout.download(np.float64, 4), want)


def test_summary_fold_many_references(ctx):
    """bc_pileup_partials on 30 references, then ONE bc_summary_fold (two launches of up to 24
    side-by-side folds): each reference's 4 doubles equal bc_pileup + bc_summary's."""
    rng = np.random.default_rng(77)
    k = 5
    nf, nf2 = norm_factors(k)
    keep, lens, works, outs, expect = [], [], [], [], []
    for i in range(30):
        L = int(rng.choice([700, 8192, 8192 * 3 + 11, 40_000, 150_000]))
        b = random_batch(rng, L, int(rng.integers(50, 3000)))
        r = D.DeviceReads(ctx, b)
        bufs = [ctx.alloc(max(8, x)) for x in (4 * k * L, 4 * L, 8 * L, 8 * L)]
        work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        ctx.pileup_partials(r, L, 0, k, nf, nf2, bufs[0].ptr, bufs[1].ptr, None, bufs[2].ptr,
                            bufs[3].ptr, work.ptr)
        keep.append((r, bufs, work, dout))
        lens.append(L)
        works.append(work.ptr)
        outs.append(dout.ptr)
        w2, d2 = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        ctx.summary(bufs[1].ptr, bufs[2].ptr, L, w2.ptr, d2.ptr)
        expect.append(d2.download(np.float64, 4))
    ctx.summary_fold(lens, works, outs)
    assert ctx.range_error() == -1
    for (r, bufs, work, dout), e in zip(keep, expect):
        assert np.array_equal(dout.download(np.float64, 4), e)


@pytest.mark.parametrize("graph", [False, True])
def test_ctx_wait_fork_join(ctx, graph):
    """References spread over three contexts' streams, forked from and joined back into the main
    context with bc_ctx_wait (eagerly, and captured into one graph begun on the main context):
    every reference's outputs and the main context's fold equal single-stream results."""
    rng = np.random.default_rng(78)
    k = 5
    nf, nf2 = norm_factors(k)
    sides = [D.Context(ctx.device), D.Context(ctx.device)]
    ctxs = [ctx] + sides
    refs = []
    for i in range(9):
        L = int(rng.choice([8192 * 3 + 11, 40_000, 150_000]))
        b = random_batch(rng, L, int(rng.integers(200, 4000)))
        r = D.DeviceReads(ctx, b)
        bufs = [ctx.alloc(max(8, x)) for x in (4 * k * L, 4 * L, 8 * L, 8 * L)]
        work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        exp, _ = O.bcount(L, 0, b)
        refs.append((L, r, bufs, work, dout, exp))

    def step():
        for s in sides:
            s.wait(ctx)
        for i, (L, r, bufs, work, dout, _) in enumerate(refs):
            ctxs[i % 3].pileup_partials(r, L, 0, k, nf, nf2, bufs[0].ptr, bufs[1].ptr, None, bufs[2].ptr,
                                        bufs[3].ptr, work.ptr)
        for s in sides:
            ctx.wait(s)
        ctx.summary_fold([x[0] for x in refs], [x[3].ptr for x in refs], [x[4].ptr for x in refs])

    if graph:
        g = ctx.capture(step)
        g.launch()
        g.launch()  # a replay over the same buffers gives the same results
    else:
        step()
    ctx.sync()
    for c in ctxs:
        assert c.range_error() == -1
    for L, r, bufs, work, dout, exp in refs:
        cnt = bufs[0].download(np.int32, k * L).reshape(k, L)
        cov = bufs[1].download(np.int32, L)
        ent = bufs[2].download(np.float64, L)
        assert np.array_equal(cnt, exp[:, :k].T.astype(np.int32))
        ocov, _, oent, _ = O.stats(exp, False)
        assert np.array_equal(cov, ocov) and np.array_equal(ent, oent)
        w2, d2 = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        ctx.summary(bufs[1].ptr, bufs[2].ptr, L, w2.ptr, d2.ptr)
        assert np.array_equal(dout.download(np.float64, 4), d2.download(np.float64, 4))


def test_cli_timing_report_keeps_stdout(golden, manifest, tmp_path):
    """BASECOUNT_HIP_TIMING=1: kernel times and the wall time on stderr, stdout still
    byte-identical to the reference's."""
    c = manifest["c1_default"]
    env = dict(os.environ, PYTHONPATH=REPO, PYTHONHASHSEED="0", BASECOUNT_HIP_TIMING="1")
    p = subprocess.run([sys.executable, "-m", "basecount_amd", c["bam"]] + c["args"], cwd=golden,
                       env=env, capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    with open(os.path.join(golden, c["stdout"]), "rb") as fh:
        assert p.stdout == gzip.decompress(fh.read())
    err = p.stderr.decode()
    assert ("kernel pileup" in err or "kernel solo" in err) and " launches, " in err and "wall " in err
