"""Sharded decode: each rank inflates and decodes only the byte range of the file
that holds its references' records.  bcio_find_ref_start finds the split points without inflating
the file (bisection over BGZF blocks, record-chain synchronisation); range streams decode
[begin, end) and fail when the record chain does not land exactly on `end`.  CPU only."""
import numpy as np
import pytest

from basecount_amd import synth
from basecount_amd.bam import BamFile, BamStream, find_ref_start
from basecount_amd.dist import shard_contiguous

CONTIGS = [("c0", 30_000), ("c1", 5_000), ("c2", 80_000), ("c3", 12_000), ("c4", 50_000), ("c5", 9_000)]


def _whole(path):
    with BamFile(path) as f:
        return f.tid.copy(), f.pos.copy(), f.cigar.copy(), f.seq.copy()


def _ranges(path, cuts, batch=5000):
    """Decode each rank's range; (per-rank arrays, whether every record is in the rank's refIDs)."""
    nref = len(cuts) - 1
    out, inside = [], True
    with BamFile(path) as f:
        n_refs = len(f.references)
    for r in range(len(cuts) - 1):
        last = r == nref - 1
        beg = find_ref_start(path, cuts[r])
        end = None if last else find_ref_start(path, cuts[r + 1])
        if beg is None or (end is not None and end <= beg):
            beg = end = None
        hi = n_refs if last else cuts[r + 1]
        parts = []
        with BamStream(path, voff_range=(beg, end)) as s:
            for b in s.batches(batch):
                t = b.tid
                inside &= not bool(np.any(((t < cuts[r]) | (t >= hi)) & (t != -1)))
                parts.append((t.copy(), b.pos.copy(), b.cigar.copy(), b.seq.copy()))
        out.append(parts)
    return out, inside


@pytest.fixture(scope="module")
def grouped_bam(tmp_path_factory):
    rs = synth.make_reads(CONTIGS, 6_000, True, 11)
    p = str(tmp_path_factory.mktemp("sd") / "grouped.bam")
    synth.write_bam(rs, p)
    return p


@pytest.mark.parametrize("world", [2, 3, 4, 6, 9])
def test_ranges_partition_a_grouped_file(grouped_bam, world):
    tid, pos, cig, seq = _whole(grouped_bam)
    cuts = shard_contiguous([L for _, L in CONTIGS], world)
    per, inside = _ranges(grouped_bam, cuts)
    assert inside
    for k, whole in enumerate((tid, pos, cig, seq)):
        got = [p[k] for parts in per for p in parts]
        assert np.array_equal(np.concatenate(got) if got else whole[:0], whole)
    # each rank holds exactly its refIDs' records
    for r, parts in enumerate(per):
        t = np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, np.int32)
        assert np.array_equal(t, tid[(tid >= cuts[r]) & (tid < cuts[r + 1])])


def test_find_ref_start_is_the_first_record_of_each_reference(tmp_path):
    """A 40 MB file: the bisection probes real block boundaries (the search is not a scan)."""
    rs = synth.make_reads(CONTIGS, 40_000, True, 12)
    p = str(tmp_path / "big.bam")
    synth.write_bam(rs, p)
    tid = _whole(p)[0]
    for t in range(len(CONTIGS) + 1):
        v = find_ref_start(p, t)
        n_before = int(np.count_nonzero(tid < t))
        if n_before == tid.size:
            assert v is None
            continue
        with BamStream(p, voff_range=(v, None)) as s:
            b = s.next_batch(10)
            assert int(b.tid[0]) == t and int(b.pos[0]) == int(rs.pos[n_before])
            b.close()


def test_unmapped_tail_goes_to_the_last_range(tmp_path):
    rs = synth.make_reads(CONTIGS[:3], 3_000, False, 13)
    n = rs.n
    um = np.arange(n) >= n - 500  # the file's last reads unmapped (refID -1), as sorted BAMs end
    rs.tid[um] = -1
    rs.pos[um] = -1
    p = str(tmp_path / "um.bam")
    synth.write_bam(rs, p)
    tid = _whole(p)[0]
    assert int(np.count_nonzero(tid == -1)) == 500
    cuts = shard_contiguous([L for _, L in CONTIGS[:3]], 2)
    per, inside = _ranges(p, cuts, batch=777)
    assert inside
    last = np.concatenate([q[0] for q in per[-1]])
    assert int(np.count_nonzero(last == -1)) == 500
    assert np.array_equal(np.concatenate([q[0] for parts in per for q in parts]), tid)
    assert find_ref_start(p, 3) is not None  # the first unmapped record


def test_a_wrong_split_fails_the_range_decode(grouped_bam):
    v = find_ref_start(grouped_bam, 2)
    bad_end = v + 7  # inside a record: the chain cannot land on it
    with pytest.raises(ValueError):
        with BamStream(grouped_bam, voff_range=(find_ref_start(grouped_bam, 0), bad_end)) as s:
            for _ in s.batches(100_000):
                pass


def test_an_ungrouped_file_is_detected(tmp_path):
    rs = synth.make_reads(CONTIGS[:4], 2_000, False, 14)
    order = np.random.default_rng(3).permutation(rs.n)
    rs2 = synth.ReadSet(references=rs.references, lengths=rs.lengths, tid=rs.tid[order], pos=rs.pos[order],
                        flag=rs.flag[order], mapq=rs.mapq[order],
                        cig_off=np.concatenate([[0], np.cumsum(np.diff(rs.cig_off)[order])]).astype(np.uint64),
                        cigar=np.concatenate([rs.cigar[int(rs.cig_off[i]):int(rs.cig_off[i + 1])] for i in order]),
                        l_seq=rs.l_seq[order], seq_off=rs.seq_off,
                        seq=rs.seq.reshape(rs.n, -1)[order].reshape(-1), qual_off=rs.qual_off,
                        qual=rs.qual.reshape(rs.n, -1)[order].reshape(-1), qstart=rs.qstart[order])
    p = str(tmp_path / "mixed_order.bam")
    synth.write_bam(rs2, p)
    cuts = shard_contiguous([L for _, L in CONTIGS[:4]], 2)
    try:
        _, inside = _ranges(p, cuts)
    except ValueError:
        inside = False  # a split the record chain does not confirm
    assert not inside


def test_empty_and_whole_ranges(grouped_bam):
    with BamStream(grouped_bam, voff_range=(None, None)) as s:
        assert s.next_batch(10) is None
        assert len(s.references) == len(CONTIGS)
    tid = _whole(grouped_bam)[0]
    with BamStream(grouped_bam, voff_range=(find_ref_start(grouped_bam, 0), None)) as s:
        n = sum(b.n_records for b in s.batches(4096))
    assert n == tid.size


@pytest.mark.parametrize("weights,world,expect", [
    ([10, 1, 1, 1, 1, 1, 1, 1, 1, 1], 2, [0, 3, 10]),
    ([5], 4, [0, 1, 1, 1, 1]),
    ([], 3, [0, 0, 0, 0]),
    ([1, 1, 1, 1], 4, [0, 1, 2, 3, 4]),
])
def test_shard_contiguous(weights, world, expect):
    assert shard_contiguous(weights, world) == expect


def test_shard_contiguous_balances_grch38():
    L = [x for _, x in synth.GRCH38]
    for world in (2, 3, 4, 8):
        c = shard_contiguous(L, world)
        loads = [sum(L[c[i]:c[i + 1]]) for i in range(world)]
        assert c[0] == 0 and c[-1] == len(L) and all(a <= b for a, b in zip(c, c[1:]))
        assert max(loads) <= 1.25 * sum(L) / world + max(L)


def test_find_record_inside_a_reference(tmp_path):
    """bcio_find_record: the first record at or past (tid, pos) splits one reference's reads."""
    rs = synth.make_reads([("one", 29_903)], 60_000, True, 15)
    p = str(tmp_path / "one.bam")
    synth.write_bam(rs, p)
    tid, pos, _, _ = _whole(p)
    for q in (1, 7_475, 14_951, 22_427, 29_000, 40_000):
        v = find_ref_start(p, 0, q)
        k = int(np.count_nonzero(pos < q))  # the file is sorted: the first k records come before
        if k == tid.size:
            assert v is None
            continue
        with BamStream(p, voff_range=(v, None)) as s:
            n = sum(b.n_records for b in s.batches(1 << 20))
        assert n == tid.size - k, q


@pytest.mark.parametrize("world", [2, 3, 5])
def test_plan_ranges_split_one_reference(tmp_path, world):
    """Every requested reference small: their positions are cut into equal parts, the ranges
    partition the file and each holds a share of the reads."""
    from basecount_amd.dist import BOUND, plan_ranges

    rs = synth.make_reads([("one", 29_903)], 30_000, False, 16)
    p = str(tmp_path / "one.bam")
    synth.write_bam(rs, p)
    cuts, owner, split = plan_ranges([29_903], [True], world, 1 << 22)
    assert split == {0} and owner == {0: 0} and len(cuts) == world + 1
    counts = []
    for r in range(world):
        beg = find_ref_start(p, *cuts[r]) if cuts[r][1] != BOUND else find_ref_start(p, cuts[r][0])
        end = None if r == world - 1 else find_ref_start(p, *cuts[r + 1])
        with BamStream(p, voff_range=(beg, end)) as s:
            counts.append(sum(b.n_records for b in s.batches(1 << 20)))
    assert sum(counts) == rs.n
    assert min(counts) > 0.5 * rs.n / world


def test_plan_ranges_whole_references_when_large():
    from basecount_amd.dist import BOUND, plan_ranges

    L = [x for _, x in synth.GRCH38]
    cuts, owner, split = plan_ranges(L, [True] * len(L), 8, 1 << 22)
    assert not split and all(p == BOUND for _, p in cuts)
    assert [owner[t] for t in range(len(L))] == sorted(owner[t] for t in range(len(L)))
