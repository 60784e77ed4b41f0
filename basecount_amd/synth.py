"""Seeded synthetic read sets and BED schemes for the benchmark configurations.

  C1  1 contig 10,000 bp, 1,000 reads x 150, 150M, seed 1            (reference CPU-runnable)
  C2  1 contig 29,903 bp, 100,000 reads x 150, 150M, seed 2          (headline metric config)
  C3  29,903 bp, 1,000,000 reads, mixed CIGAR (0-5 S each end, one M/I/D/=/X block of 1-3
      inside the M run), 1% N bases, mapq U[0,60], seed 3
  C4  C3 + 98-amplicon ARTIC-style BED
  C5  24 contigs with GRCh38 chr1-22,X,Y lengths (3.09 Gb), 50,000 reads x 150 each, 150M, seed 5

Bases U{A,C,G,T}, qualities U[2,40].  Reads come out coordinate-sorted per contig (as a sorted
BAM would be) unless ``unsorted=True``.  A ``ReadSet`` holds records in BAM CSR layout and can be
written as a BGZF BAM (``write_bam``) or turned directly into per-contig GPU batches
(``batches``) without a BAM round trip.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

GRCH38 = [
    ("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
    ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
    ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
    ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
    ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
    ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415),
]

ACGT = np.array([1, 2, 4, 8], np.uint8)  # BAM 4-bit codes
CODE_N = 15

CONFIGS = {
    "c1": dict(contigs=[("ref", 10_000)], reads=1_000, mixed=False, seed=1),
    "c2": dict(contigs=[("MN908947.3", 29_903)], reads=100_000, mixed=False, seed=2),
    "c3": dict(contigs=[("MN908947.3", 29_903)], reads=1_000_000, mixed=True, seed=3),
    "c4": dict(contigs=[("MN908947.3", 29_903)], reads=1_000_000, mixed=True, seed=3, bed=True),
    "c5": dict(contigs=GRCH38, reads=50_000, mixed=False, seed=5, per_contig=True),
}


@dataclass
class ReadSet:
    references: list
    lengths: list
    tid: np.ndarray      # int32 [n]
    pos: np.ndarray      # int32 [n]
    flag: np.ndarray     # uint16 [n]
    mapq: np.ndarray     # uint8 [n]
    cig_off: np.ndarray  # uint64 [n+1]
    cigar: np.ndarray    # uint32 BAM words
    l_seq: np.ndarray    # int32 [n]
    seq_off: np.ndarray  # uint64 [n+1] (bytes)
    seq: np.ndarray      # uint8 packed
    qual_off: np.ndarray  # uint64 [n+1]
    qual: np.ndarray     # uint8
    qstart: np.ndarray   # int32 [n] leading soft clip

    @property
    def n(self) -> int:
        return int(self.tid.size)


def _cig(op: int, ln) -> np.ndarray:
    return (np.asarray(ln, np.uint32) << 4) | np.uint32(op)


def make_reads(contigs, reads_per_contig: int, mixed: bool, seed: int, read_len: int = 150,
               unsorted: bool = False, n_frac: float = 0.01) -> ReadSet:
    rng = np.random.default_rng(seed)
    tids, poss, cigs, ncig, qstarts, mapqs = [], [], [], [], [], []
    for t, (_, L) in enumerate(contigs):
        n = reads_per_contig
        if not mixed:
            span = np.full(n, read_len, np.int64)
            cig = np.broadcast_to(_cig(0, read_len), (n, 1)).copy()
            nc = np.ones(n, np.int64)
            qs = np.zeros(n, np.int32)
        else:
            a = rng.integers(0, 6, n)           # leading soft clip
            b = rng.integers(0, 6, n)           # trailing soft clip
            kind = rng.integers(0, 5, n)        # 0 M, 1 I, 2 D, 3 =, 4 X
            blen = rng.integers(1, 4, n)
            core = read_len - a - b             # query bases inside the alignment
            qcons = np.where(kind == 2, 0, blen)  # block's query consumption
            m_tot = core - qcons
            m1 = (rng.random(n) * (m_tot - 1)).astype(np.int64) + 1  # >= 1 on both sides
            m2 = m_tot - m1
            ops = np.stack([np.full(n, 4), np.zeros(n, np.int64), np.array([0, 1, 2, 7, 8])[kind],
                            np.zeros(n, np.int64), np.full(n, 4)], 1)
            lens = np.stack([a, m1, blen, m2, b], 1)
            keep = lens > 0
            words = (lens.astype(np.uint32) << 4) | ops.astype(np.uint32)
            nc = keep.sum(1)
            # compact rows (drop zero-length soft clips)
            order = np.argsort(~keep, axis=1, kind="stable")
            cig = np.take_along_axis(words, order, 1)
            span = m1 + m2 + np.where((kind == 0) | (kind >= 2), blen, 0)
            qs = a.astype(np.int32)
        start = rng.integers(0, max(1, L - span.max() + 1), n)
        if not unsorted:
            o = np.argsort(start, kind="stable")
            start, cig, nc, qs = start[o], cig[o], nc[o], qs[o]
        tids.append(np.full(n, t, np.int32))
        poss.append(start.astype(np.int32))
        cigs.append((cig, nc))
        qstarts.append(qs)
        mapqs.append(rng.integers(0, 61, n).astype(np.uint8) if mixed else np.full(n, 60, np.uint8))
    tid = np.concatenate(tids)
    pos = np.concatenate(poss)
    qstart = np.concatenate(qstarts)
    mapq = np.concatenate(mapqs)
    nc = np.concatenate([c[1] for c in cigs])
    width = max(c[0].shape[1] for c in cigs)
    mat = np.concatenate([np.pad(c[0], ((0, 0), (0, width - c[0].shape[1]))) for c in cigs])
    cig_off = np.zeros(tid.size + 1, np.uint64)
    np.cumsum(nc, out=cig_off[1:])
    cigar = mat[np.arange(width)[None, :] < nc[:, None]].astype(np.uint32)
    n = tid.size
    codes = ACGT[rng.integers(0, 4, (n, read_len))]
    if mixed and n_frac > 0:
        codes[rng.random((n, read_len)) < n_frac] = CODE_N
    if read_len % 2:  # odd length: the last byte's low nibble is padding (0)
        codes = np.pad(codes, ((0, 0), (0, 1)))
    packed = ((codes[:, 0::2] << 4) | codes[:, 1::2]).astype(np.uint8)
    qual = rng.integers(2, 41, (n, read_len)).astype(np.uint8)
    nb = (read_len + 1) // 2
    return ReadSet(
        references=[c[0] for c in contigs], lengths=[int(c[1]) for c in contigs],
        tid=tid, pos=pos, flag=np.zeros(n, np.uint16), mapq=mapq, cig_off=cig_off, cigar=cigar,
        l_seq=np.full(n, read_len, np.int32),
        seq_off=np.arange(n + 1, dtype=np.uint64) * np.uint64(nb), seq=packed.reshape(-1),
        qual_off=np.arange(n + 1, dtype=np.uint64) * np.uint64(read_len),
        qual=qual.reshape(-1), qstart=qstart,
    )


def make_config(name: str, unsorted: bool = False, contigs=None, reads=None) -> ReadSet:
    c = CONFIGS[name.lower()]
    if c.get("per_contig"):  # each contig's reads from its own seed (contig_reads)
        cs = list(contigs or c["contigs"])
        return contig_reads(cs, range(len(cs)), reads or c["reads"], c["mixed"], c["seed"], unsorted=unsorted)
    return make_reads(contigs or c["contigs"], reads or c["reads"], c["mixed"], c["seed"],
                      unsorted=unsorted)


def contig_reads(contigs, indices, reads_per_contig: int, mixed: bool, seed: int, unsorted: bool = False) -> ReadSet:
    """The reads of contigs[i] for i in `indices`, each contig from its own seed (seed + 1000003 i),
    so a contig's reads do not depend on which others are generated with it: a rank holding a
    shard of the contigs (bench.py, several GPUs) counts exactly the reads one process would."""
    parts = [make_reads([contigs[i]], reads_per_contig, mixed, seed + 1000003 * i, unsorted=unsorted)
             for i in indices]
    return concat(parts, [contigs[i][0] for i in indices], [int(contigs[i][1]) for i in indices])


def concat(parts, references, lengths) -> ReadSet:
    """One ReadSet of several (part k's reads on contig k)."""
    if not parts:
        z = lambda dt: np.zeros(0, dt)  # noqa: E731
        return ReadSet(references=[], lengths=[], tid=z(np.int32), pos=z(np.int32), flag=z(np.uint16),
                       mapq=z(np.uint8), cig_off=np.zeros(1, np.uint64), cigar=z(np.uint32), l_seq=z(np.int32),
                       seq_off=np.zeros(1, np.uint64), seq=z(np.uint8), qual_off=np.zeros(1, np.uint64),
                       qual=z(np.uint8), qstart=z(np.int32))
    tid = np.concatenate([np.full(p.n, k, np.int32) for k, p in enumerate(parts)])

    def offs(name):
        out, base = [np.zeros(1, np.uint64)], np.uint64(0)
        for p in parts:
            o = getattr(p, name)
            out.append(o[1:] + base)
            base += o[-1]
        return np.concatenate(out).astype(np.uint64)

    cat = lambda name: np.concatenate([getattr(p, name) for p in parts])  # noqa: E731
    return ReadSet(references=list(references), lengths=list(lengths), tid=tid, pos=cat("pos"), flag=cat("flag"),
                   mapq=cat("mapq"), cig_off=offs("cig_off"), cigar=cat("cigar"), l_seq=cat("l_seq"),
                   seq_off=offs("seq_off"), seq=cat("seq"), qual_off=offs("qual_off"), qual=cat("qual"),
                   qstart=cat("qstart"))


def subset(rs: ReadSet, order) -> ReadSet:
    """The reads of `rs` in the given order (an index array: reorders, drops or repeats records),
    e.g. a file whose references are interleaved.  Reads are fixed-length (make_reads)."""
    order = np.asarray(order, np.int64)
    nc = np.diff(rs.cig_off.astype(np.int64))[order]
    L = int(rs.seq_off[1] - rs.seq_off[0]) if rs.n else 0
    Q = int(rs.qual_off[1] - rs.qual_off[0]) if rs.n else 0
    return ReadSet(references=rs.references, lengths=rs.lengths, tid=rs.tid[order], pos=rs.pos[order],
                   flag=rs.flag[order], mapq=rs.mapq[order],
                   cig_off=np.concatenate([[0], np.cumsum(nc)]).astype(np.uint64),
                   cigar=np.concatenate([rs.cigar[int(rs.cig_off[i]):int(rs.cig_off[i + 1])] for i in order])
                   if order.size else rs.cigar[:0],
                   l_seq=rs.l_seq[order], seq_off=(np.arange(order.size + 1) * L).astype(np.uint64),
                   seq=rs.seq.reshape(rs.n, -1)[order].reshape(-1),
                   qual_off=(np.arange(order.size + 1) * Q).astype(np.uint64),
                   qual=rs.qual.reshape(rs.n, -1)[order].reshape(-1), qstart=rs.qstart[order])


def write_bam(rs: ReadSet, path: str, level: int = 1) -> None:
    from .bam import write_bam as _w

    _w(path, rs.references, rs.lengths, rs.tid, rs.pos, rs.flag, rs.mapq, rs.cig_off, rs.cigar,
       rs.l_seq, rs.seq_off, rs.seq, rs.qual_off, rs.qual, level=level)


def artic_bed(n_tiles: int = 98, first: int = 30, stride: int = 300, amp: int = 400, plen: int = 22,
              chrom: str = "MN908947.3", scheme: str = "nCoV-2019") -> str:
    """ARTIC-style primer BED: <scheme>_<tile>_LEFT/RIGHT, an extra _alt LEFT every 10th tile."""
    lines = []
    for i in range(1, n_tiles + 1):
        s = first + (i - 1) * stride
        e = s + amp
        pool = 1 if i % 2 else 2
        lines.append(f"{chrom}\t{s}\t{s + plen}\t{scheme}_{i}_LEFT\t{pool}\t+")
        if i % 10 == 0:
            lines.append(f"{chrom}\t{s + 5}\t{s + 5 + plen}\t{scheme}_{i}_LEFT_alt\t{pool}\t+")
        lines.append(f"{chrom}\t{e - plen}\t{e}\t{scheme}_{i}_RIGHT\t{pool}\t-")
    return "\n".join(lines) + "\n"


def batch_arrays(rs: ReadSet, t: int, mmq: int = 0) -> dict:
    """Accepted reads of contig t in the bc_reads layout (host numpy arrays)."""
    sel = (rs.tid == t) & ((rs.flag & 4) == 0) & (rs.mapq.astype(np.int64) >= mmq)
    idx = np.nonzero(sel)[0]
    return dict(
        pos=rs.pos[idx].astype(np.int32),
        cig_beg=rs.cig_off[:-1][idx].astype(np.uint32),
        cig_n=(rs.cig_off[1:] - rs.cig_off[:-1])[idx].astype(np.uint32),
        seq_nib=(2 * rs.seq_off[:-1][idx] + rs.qstart[idx].astype(np.uint64)).astype(np.uint32),
        cigar=rs.cigar, seq=rs.seq, qual=_nibble_qual(rs),
    )


def _nibble_qual(rs: ReadSet) -> np.ndarray:
    """QUAL re-laid by nibble index (base i of record r at 2*seq_off[r] + i)."""
    if rs.l_seq.size and np.all(rs.l_seq % 2 == 0) and np.all(
            rs.qual_off[:-1] == 2 * rs.seq_off[:-1]):
        return rs.qual
    out = np.full(2 * int(rs.seq_off[-1]), 0xFF, np.uint8)
    for r in range(rs.n):
        a, b = int(rs.qual_off[r]), int(rs.qual_off[r + 1])
        d = 2 * int(rs.seq_off[r])
        out[d: d + (b - a)] = rs.qual[a:b]
    return out


def ref_events(rs: ReadSet, t: int | None = None) -> int:
    """Reference-consuming CIGAR events (M/=/X/D/N bases) = 'bases piled' for Gbases/s."""
    w = rs.cigar
    op = w & 0xF
    ln = (w >> 4).astype(np.int64)
    cons = (op == 0) | (op == 2) | (op == 3) | (op == 7) | (op == 8)
    if t is None:
        return int(ln[cons].sum())
    nc = (rs.cig_off[1:] - rs.cig_off[:-1]).astype(np.int64)
    rec = np.repeat(np.arange(rs.n), nc)
    return int(ln[cons & (rs.tid[rec] == t)].sum())
