"""Host components of the path on CPU: BAM writer -> decoder round trip, read selection
(main.py:141-174), the byte-exact TSV formatter (main.py:454-466), the bcount adapter's argument
errors (pybind11 TypeError text), the CLI surface, and the BED scheme parser."""
import io
import math
import os
from contextlib import redirect_stdout

import numpy as np
import pytest

from basecount_amd import fmt, synth
from basecount_amd.bam import BamFile
from basecount_amd.main import build_parser
from basecount_amd.scheme import load_scheme

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def mixed_bam(tmp_path_factory):
    rs = synth.make_reads([("chrA", 3_000), ("chrB", 1_200), ("chrC", 500)], 700, True, 17)
    # mark some reads unmapped to exercise the filter
    rs.flag[::13] |= 4
    path = str(tmp_path_factory.mktemp("bam") / "mixed.bam")
    synth.write_bam(rs, path)
    return rs, path


def test_bam_round_trip(mixed_bam):
    rs, path = mixed_bam
    with BamFile(path) as f:
        assert list(f.references) == rs.references and list(f.lengths) == rs.lengths
        assert f.n_records == rs.n
        assert np.array_equal(f.tid, rs.tid) and np.array_equal(f.pos, rs.pos)
        assert np.array_equal(f.mapq, rs.mapq) and np.array_equal(f.flag, rs.flag)
        assert np.array_equal(f.cig_off, rs.cig_off) and np.array_equal(f.cigar, rs.cigar)
        assert np.array_equal(f.l_seq, rs.l_seq)
        assert np.array_equal(f.seq, rs.seq)
        assert np.array_equal(f.qstart, rs.qstart)
        assert not f.rec_err.any()


@pytest.mark.parametrize("mmq", [0, 30, 60])
def test_select_matches_numpy(mixed_bam, mmq):
    """main.py:165: keep `not is_unmapped and mapping_quality >= mmq`, grouped by reference."""
    rs, path = mixed_bam
    with BamFile(path) as f:
        want = [True, False, True]
        sel = f.select(mmq, want)
        keep = ((rs.flag & 4) == 0) & (rs.mapq >= mmq) & np.isin(rs.tid, [0, 2])
        idx = np.nonzero(keep)[0]
        order = np.argsort(rs.tid[idx], kind="stable")
        idx = idx[order]
        assert np.array_equal(sel.pos, rs.pos[idx])
        assert np.array_equal(sel.cig_beg, rs.cig_off[:-1][idx].astype(np.uint32))
        assert np.array_equal(sel.cig_n, np.diff(rs.cig_off)[idx].astype(np.uint32))
        assert np.array_equal(sel.seq_nib, (2 * rs.seq_off[:-1][idx] + rs.qstart[idx]).astype(np.uint32))
        counts = [int(((rs.tid[idx]) == t).sum()) for t in range(3)]
        assert list(np.diff(sel.ref_beg)) == counts


def _python_rows(ref, counts, pc, ent, sec, dp, long_format):
    return fmt._rows_text_py(ref, counts, pc, ent, sec, dp, long_format)


@pytest.mark.parametrize("dp", [0, 1, 3, 5, 7, 12])
@pytest.mark.parametrize("long_format", [False, True])
def test_formatter_matches_python_round(dp, long_format):
    """bcio_fmt_rows (C++) vs str(round(x, dp)) exactly as main.py:454-466 prints rows."""
    rng = np.random.default_rng(dp + 100 * long_format)
    k, L = 5, 400
    counts = rng.integers(0, 40, (k, L)).astype(np.int32)
    counts[:, ::7] = 0           # zero coverage: ints -1 / 1 / 1
    counts[1:, 3::11] = 0        # one non-zero column: secondary entropy is int 1
    cov = counts.sum(0)
    with np.errstate(invalid="ignore", divide="ignore"):
        pc = np.where(cov > 0, 100.0 * (counts / np.maximum(cov, 1)), -1.0)
    ent = rng.random(L)
    sec = rng.random(L)
    # rounding ties and awkward magnitudes
    specials = [0.5, 0.25, 0.125, 0.0625, 2.675, 1.005, 1e-5, 1e-16, 123456.789, 99.99999999, 1 / 3, 2 / 3]
    ent[: len(specials)] = specials
    sec[: len(specials)] = specials[::-1]
    got = fmt.rows_text("chré", counts, pc, ent, sec, dp, long_format)
    exp = _python_rows("chré", counts, pc, ent, sec, dp, long_format)
    assert got == exp


def test_pyround_native_matches_python():
    rng = np.random.default_rng(3)
    xs = list(rng.random(2000) * 10.0 ** rng.integers(-8, 8, 2000)) + [0.5, 1.5, 2.5, -0.0, 1e300, 5e-324]
    for dp in (0, 2, 3, 6):
        for x in xs:
            assert fmt.pyround_native(float(x), dp) == str(round(float(x), dp)), (x, dp)


@pytest.mark.parametrize("args", [
    (None, 0, [], [], [], []),
    (10, -1, [], [], [], []),
    (10, 0, ["A"], [None], [0], [[(0, 1)]]),
    (10, 0, ["A"], [[30]], [-1], [[(0, 1)]]),
    (10, 0, [b"A"], [[30]], [0], [[(0, 1)]]),
    (10, 0, ["A"], [[30]], [0], [None]),
    (2 ** 32, 0, [], [], [], []),
])
def test_bcount_adapter_type_errors(args):
    """count.cpp:102-105 through pybind11: unconvertible arguments raise TypeError (before any
    device work)."""
    from basecount_amd.count import bcount

    with pytest.raises(TypeError) as ei:
        bcount(*args)
    assert str(ei.value).startswith("bcount(): incompatible function arguments.")
    assert "Invoked with: " in str(ei.value)


def test_cli_help_and_version(monkeypatch):
    """main.py:379-431: the reference's flags and help (argparse of Python 3.10, 80 columns)."""
    monkeypatch.setenv("COLUMNS", "80")
    text = build_parser().format_help()
    for flag in ("--references", "--min-base-quality", "--min-mapping-quality", "--chunk-size",
                 "--show-n-bases", "--long-format", "--summarise", "--summarise-with-bed",
                 "--decimal-places", "-v, --version"):
        assert flag in text
    assert text.startswith("usage: basecount [-h] [-v]")
    assert "Path to BAM file (an index file is not required)" in text
    out = io.StringIO()
    with redirect_stdout(out), pytest.raises(SystemExit):
        build_parser().parse_args(["-v"])
    assert out.getvalue().strip() == "1.7.2"


def test_scheme_windows():
    """scheme.py:60-74: inner windows clipped to the neighbours' primers, sorted by tile."""
    tiles = load_scheme(os.path.join(HERE, "golden", "scheme.bed"))
    assert len(tiles) == 98
    nums = [int(t[1]) for t in tiles]
    assert nums == sorted(nums)
    for i, (_, _, w) in enumerate(tiles):
        assert w["start"] <= w["inside_start"] <= w["inside_end"] <= w["end"] or i == 0
        if i > 0:
            assert w["inside_start"] == tiles[i - 1][2]["end"]
        if i + 1 < len(tiles):
            assert w["inside_end"] == tiles[i + 1][2]["start"]
    raw = load_scheme(os.path.join(HERE, "golden", "scheme.bed"), clip=False)
    assert [t[1] for t in raw] == [t[1] for t in tiles]


def test_synth_event_checksum():
    """ref_events = sum of M/=/X/D/N lengths (the 'bases piled' of Gbases/s)."""
    rs = synth.make_reads([("a", 5_000)], 300, True, 4)
    cig = rs.cigar
    ops, lens = cig & 15, cig >> 4
    assert synth.ref_events(rs) == int(lens[np.isin(ops, [0, 2, 3, 7, 8])].sum())
    assert math.isclose(synth.ref_events(rs) / 300, 150, rel_tol=0.1)


@pytest.mark.parametrize("inflater", ["libdeflate", "zlib"])
def test_bam_odd_length_quals(tmp_path, monkeypatch, inflater):
    """QUAL lands at nibble index 2*seq_off + i with the pad byte of an odd-length read = 0xFF
    (the decoder leaves no byte of its output arrays unwritten); both inflaters agree."""
    if inflater == "zlib":
        monkeypatch.setenv("BCIO_ZLIB", "1")
    rs = synth.make_reads([("chrA", 2_000), ("chrB", 900)], 300, True, 23, read_len=151)
    path = str(tmp_path / "odd.bam")
    synth.write_bam(rs, path)
    with BamFile(path) as f:
        assert np.array_equal(f.seq, rs.seq)
        assert np.array_equal(f.qual, synth._nibble_qual(rs))
        assert np.array_equal(f.l_seq, rs.l_seq)


def test_bam_corrupt_block(tmp_path):
    """A damaged deflate stream is an error, not a silently short read set."""
    rs = synth.make_reads([("chrA", 2_000)], 200, False, 5)
    path = str(tmp_path / "bad.bam")
    synth.write_bam(rs, path)
    data = bytearray(open(path, "rb").read())
    mid = len(data) // 2
    data[mid: mid + 64] = bytes(64)
    open(path, "wb").write(bytes(data))
    with pytest.raises(Exception):
        BamFile(path)


@pytest.mark.parametrize("dp", [0, 1, 2, 3, 4, 5])
def test_pyround_native_decimal_ties(dp):
    """Values at and next to decimal ties (k + 1/2)·10^-dp, whose binary value sits just above or
    below the tie: the long-double fast path (dp <= 4) and printf/strtod (dp > 4) both match
    CPython's round()."""
    rng = np.random.default_rng(dp)
    ks = rng.integers(0, 10 ** 7, 3000)
    xs = []
    for kk in ks:
        t = (int(kk) + 0.5) / 10 ** dp
        xs += [t, np.nextafter(t, 0.0), np.nextafter(t, 1e300), -t]
    xs += [float(v) / 8 for v in range(-64, 64)] + [2.0 ** 52 + 0.5, 2.0 ** 53, 4.5e15, 9.5e15]
    for x in xs:
        assert fmt.pyround_native(float(x), dp) == str(round(float(x), dp)), (x, dp)


def test_select_multi_chunk(tmp_path):
    """The parallel selection (65,536-record chunks) keeps file order per reference, the global
    accepted ordinals, the first KeyError read (main.py:166) and the decoder's reference spans."""
    rs = synth.make_reads([("a", 40_000), ("b", 30_000), ("c", 20_000)], 60_000, True, 31)
    rs.flag[::7] |= 4
    path = str(tmp_path / "big.bam")
    synth.write_bam(rs, path)
    with BamFile(path) as f:
        ops, lens = f.cigar & 15, (f.cigar >> 4).astype(np.int64)
        cons = np.isin(ops, [0, 2, 3, 7, 8])
        rec_of = np.repeat(np.arange(f.n_records), np.diff(f.cig_off).astype(np.int64))
        span = np.bincount(rec_of, weights=np.where(cons, lens, 0), minlength=f.n_records)
        assert np.array_equal(f.ref_span, span.astype(np.int64))
        for mmq in (0, 31):
            sel = f.select(mmq, [True, False, True])
            acc = ((rs.flag & 4) == 0) & (rs.mapq >= mmq)
            ordinal = np.cumsum(acc) - 1
            keep = acc & np.isin(rs.tid, [0, 2])
            idx = np.nonzero(keep)[0]
            idx = idx[np.argsort(rs.tid[idx], kind="stable")]
            assert np.array_equal(sel.rec, idx)
            assert np.array_equal(sel.ordinal, ordinal[idx])
            assert np.array_equal(sel.span, span[idx].astype(np.int64))
            assert sel.n_accepted == int(acc.sum())
            bad = np.nonzero(acc & (rs.tid == 1))[0]
            assert sel.keyerror_rec == bad[0] and sel.keyerror_ordinal == ordinal[bad[0]]


def _event_numpy(seq: np.ndarray) -> np.ndarray:
    """BC_SEQ_EVENT restated in numpy (basecount_hip.h): byte m = class(base 2m) | class(2m+1)
    << 4 with A 1, C 2, G 4, T 8, N 3 and every other code 0."""
    cls = np.zeros(16, np.uint8)
    cls[[1, 2, 4, 8, 15]] = [1, 2, 4, 8, 3]
    return cls[seq >> 4] | (cls[seq & 15] << 4)


def test_decoder_emits_event_layout(mixed_bam):
    """The decoder fills the kernels' sequence layout while decoding (no device
    conversion pass per batch): identical to the standalone converter and to the restatement,
    zero-padded to bc_seq_event_bytes."""
    from basecount_amd.bam import seq_event_bytes, seq_to_event

    rs, path = mixed_bam
    with BamFile(path) as f:
        n = f.seq.size
        assert f.seq_event.size == seq_event_bytes(n) == (n + 15) // 16 * 16 + 16
        assert np.array_equal(f.seq_event[:n], _event_numpy(f.seq))
        assert not f.seq_event[n:].any()
        assert np.array_equal(seq_to_event(f.seq, nthreads=3), f.seq_event)
    every = np.arange(256, dtype=np.uint8)
    assert np.array_equal(seq_to_event(every)[:256], _event_numpy(every))
    assert seq_to_event(np.zeros(0, np.uint8)).tolist() == [0] * 16
