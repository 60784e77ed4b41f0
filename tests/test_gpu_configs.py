"""The BASELINE configurations at full size through the product path, against the oracle
(no config may stay untested on the GPU).

  C5  24 GRCh38-sized contigs (3.09 Gb) x 50,000 reads: every contig through bc_pileup +
      bc_summary (the sparse k_pileup_solo shape), one test per contig: coverage sum == events
      piled, counts exact and coverage / entropies / secondary entropies bit-identical to the
      oracle at every position of all 24 (3.09 G positions); then the CLI's --summarise over a
      written BAM == the oracle's main.py:469-499 text for all 24.
  C4  1,000,000 mixed-CIGAR reads + the 98-amplicon BED through the CLI's --summarise-with-bed
      (the deep k_rc -> k_stats -> k_sum -> k_amplicon chain) == main.py:469-595 from the oracle.
  C3  the same reads through the CLI's default per-position rows == main.py:454-466 from the
      oracle, byte for byte.
"""
import contextlib
import io
import os

import numpy as np
import pytest

import oracle as O
from basecount_amd import device as D
from basecount_amd import synth
from basecount_amd.bam import BamFile, seq_to_event
from basecount_amd.main import norm_factors
from basecount_amd.scheme import load_scheme

pytestmark = pytest.mark.gpu
T = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def ctx():
    return D.Context(0)


def _run_cli(argv):
    from basecount_amd.main import run

    buf = io.BytesIO()
    txt = io.TextIOWrapper(buf, encoding="utf-8", write_through=True)
    with contextlib.redirect_stdout(txt):
        run(argv)
        txt.flush()
    return buf.getvalue().decode()


@pytest.fixture(scope="module")
def c5():
    return synth.make_config("c5")


@pytest.fixture(scope="module")
def c5_event(c5):
    return seq_to_event(c5.seq)


@pytest.mark.parametrize("t", range(len(synth.GRCH38)), ids=[n for n, _ in synth.GRCH38])
def test_c5_contig(ctx, c5, c5_event, t):
    rs = c5
    k = 5
    nf, nf2 = norm_factors(k)
    name, L = rs.references[t], rs.lengths[t]
    b = synth.batch_arrays(rs, t, 0)
    r = D.DeviceReads(ctx, dict(b, seq_event=c5_event))
    bufs = [ctx.alloc(n) for n in (4 * k * L, 4 * L, 8 * L, 8 * L, D.summary_work_bytes(L), 32)]
    counts, cov, ent, sec, work, out = bufs
    try:
        ctx.pileup(r, L, 0, k, nf, nf2, counts.ptr, cov.ptr, None, ent.ptr, sec.ptr)
        ctx.summary(cov.ptr, ent.ptr, L, work.ptr, out.ptr)
        assert ctx.range_error() == -1
        hcov = cov.download(np.int32, L)
        hent = ent.download(np.float64, L)
        s = out.download(np.float64, 4)
        # checksum of checksums: all-M reads without N put every event into the coverage
        assert int(hcov.sum(dtype=np.int64)) == synth.ref_events(rs, t)
        c64 = hcov.astype(np.int64)
        assert s[0] == np.mean(c64) and s[1] == np.mean(hent)
        assert int(s[2]) == int(np.count_nonzero(hcov))
        del c64
        exp, (br, _) = O.bcount(L, 0, b)
        assert br == -1
        got = counts.download(np.int32, k * L).reshape(k, L)
        assert np.array_equal(got, exp[:, :k].T)
        del got
        ocov, opc, oent, osec = O.stats(exp, False, nthreads=T)
        del opc, exp
        assert np.array_equal(hcov, ocov)
        assert np.array_equal(hent, oent)  # bit-identical (glibc log2 on the device)
        assert np.array_equal(sec.download(np.float64, L), osec)
    finally:
        for x in bufs:
            x.free()
        r.free()


def test_c5_summary_only_per_contig(ctx, c5, c5_event):
    """the summary-only sweep (bc_pileup_summary with no per-position outputs,
    what --summarise needs) on every C5 contig: the same four numbers as numpy over the oracle's
    per-position coverage and entropies (main.py:469-499)."""
    k = 5
    nf, nf2 = norm_factors(k)
    for t, name in enumerate(c5.references):
        L = c5.lengths[t]
        b = synth.batch_arrays(c5, t, 0)
        r = D.DeviceReads(ctx, dict(b, seq_event=c5_event))
        work, out = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
        try:
            ctx.pileup_summary(r, L, 0, k, nf, nf2, None, None, None, None, None, work.ptr, out.ptr)
            assert ctx.range_error() == -1
            s = out.download(np.float64, 4)
            exp, (br, _) = O.bcount(L, 0, b)
            assert br == -1
            ocov, _, oent, _ = O.stats(exp, False, nthreads=T)
            del exp
            # main.py:469-499's numbers: np.mean of the coverages and entropies, the covered count
            assert s[0] == np.mean(ocov.astype(np.int64)) and s[1] == np.mean(oent), name
            assert int(s[2]) == int(np.count_nonzero(ocov)) and int(s[3]) == int(ocov.sum(dtype=np.int64))
            del ocov, oent
        finally:
            work.free()
            out.free()
            r.free()


@pytest.mark.parametrize("batch", [None, "200000"])
def test_c5_cli_summarise(c5, tmp_path, monkeypatch, batch):
    """batch 200000: the 1.2 M records stream in 6 batches; contigs cut by a batch boundary are
    accumulated (bc_count per batch) and finished by kernel 2, the others take the fused sweep."""
    if batch:
        monkeypatch.setenv("BASECOUNT_BATCH_RECORDS", batch)
    bam = str(tmp_path / "c5.bam")
    synth.write_bam(c5, bam)
    got = _run_cli([bam, "--summarise"])
    _, blocks = O.split_blocks(got, True)
    assert sorted(blocks) == sorted(c5.references)
    with BamFile(bam) as f:
        for t, name in enumerate(f.references):
            b, n = O.batch_from_bam(f, t, 0)
            exp, (br, _) = O.bcount(f.lengths[t], 0, b)
            assert br == -1
            assert blocks[name] == O.summary_text(name, exp, False, n, 3, nthreads=T), name
            del exp


@pytest.fixture(scope="module")
def c3_bam(tmp_path_factory):
    rs = synth.make_config("c3")
    d = tmp_path_factory.mktemp("c3")
    bam = str(d / "c3.bam")
    synth.write_bam(rs, bam)
    bed = str(d / "scheme.bed")
    with open(bed, "w") as fh:
        fh.write(synth.artic_bed())
    return bam, bed


@pytest.mark.parametrize("args,mbq,mmq", [([], 0, 0),
                                          (["--min-base-quality", "20", "--min-mapping-quality", "30"], 20, 30)])
def test_c4_cli_summarise_with_bed(c3_bam, args, mbq, mmq):
    bam, bed = c3_bam
    got = _run_cli([bam, "--summarise-with-bed", bed] + args)
    tiles = [(w["inside_start"], w["inside_end"]) for _, _, w in load_scheme(bed)]
    assert len(tiles) == 98
    with BamFile(bam) as f:
        b, n = O.batch_from_bam(f, 0, mmq)
        exp, (br, _) = O.bcount(f.lengths[0], mbq, b)
        assert br == -1
        assert got == O.summary_text(f.references[0], exp, False, n, 3, tiles=tiles)


@pytest.mark.parametrize("chunk", [None, "1000"])
def test_c3_cli_rows(c3_bam, chunk):
    """--chunk-size 1000: the reference flushes every 1000 reads (main.py:142-162); here the file
    streams in 65,536-record batches (main.batch_records), 16 of them, each counted into the
    reference's accumulator by the read-chunked kernel, then kernel 2 once."""
    bam, _ = c3_bam
    got = _run_cli([bam] + (["--chunk-size", chunk] if chunk else []))
    with BamFile(bam) as f:
        b, _ = O.batch_from_bam(f, 0, 0)
        exp, (br, _) = O.bcount(f.lengths[0], 0, b)
        assert br == -1
        header = "\t".join(["reference", "position", "coverage", "num_a", "num_c", "num_g", "num_t",
                            "num_ds", "pc_a", "pc_c", "pc_g", "pc_t", "pc_ds", "entropy",
                            "secondary_entropy"]) + "\n"
        assert got == header + O.rows_text(f.references[0], exp, False, False, 3)


@pytest.mark.parametrize("batch", [None, "7000"])
def test_unsorted_bam_cli_rows(tmp_path, monkeypatch, batch):
    """An unsorted BAM (C2 shape, 3 contigs, reads in random order): the CLI takes the
    event-parallel k_count + k_stats path; rows byte-identical to the oracle's main.py:454-466.
    In 7000-record batches the contigs come back after a batch without them: the stream starts
    again accumulating every contig to the end of the file (main._Ungrouped)."""
    if batch:
        monkeypatch.setenv("BASECOUNT_BATCH_RECORDS", batch)
    rs = synth.make_reads([("u1", 29_903), ("u2", 5_000), ("u3", 70_000)], 40_000, True, 91, unsorted=True)
    order = np.random.default_rng(5).permutation(rs.n)  # interleave the contigs too
    rs2 = synth.ReadSet(references=rs.references, lengths=rs.lengths, tid=rs.tid[order], pos=rs.pos[order],
                        flag=rs.flag[order], mapq=rs.mapq[order],
                        cig_off=np.concatenate([[0], np.cumsum(np.diff(rs.cig_off)[order])]).astype(np.uint64),
                        cigar=np.concatenate([rs.cigar[int(rs.cig_off[i]):int(rs.cig_off[i + 1])] for i in order]),
                        l_seq=rs.l_seq[order], seq_off=rs.seq_off,
                        seq=rs.seq.reshape(rs.n, -1)[order].reshape(-1), qual_off=rs.qual_off,
                        qual=rs.qual.reshape(rs.n, -1)[order].reshape(-1), qstart=rs.qstart[order])
    bam = str(tmp_path / "unsorted.bam")
    synth.write_bam(rs2, bam)
    got = _run_cli([bam, "--show-n-bases", "--min-base-quality", "15"])
    header, blocks = O.split_blocks(got, False)
    with BamFile(bam) as f:
        assert sorted(blocks) == sorted(f.references)
        for t, name in enumerate(f.references):
            b, _ = O.batch_from_bam(f, t, 0)
            exp, (br, _) = O.bcount(f.lengths[t], 15, b)
            assert br == -1
            assert blocks[name] == O.rows_text(name, exp, True, False, 3), name
