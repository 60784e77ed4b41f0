"""ORACLE — test infrastructure only.  A minimal pysam stand-in so the REFERENCE's own Python
(/root/reference/basecount/main.py) can run in this container over our BAM decoder, to produce the
golden fixtures in tests/golden/ (tests/golden/make_golden.py).  Never imported by the product.

Covers exactly what main.py uses: set_verbosity (main.py:97-99), AlignmentFile(bam, mode)
(main.py:98) with .references / .lengths (main.py:86-90,122), .fetch(until_eof=True)
(main.py:127), .close() (main.py:204), and per-read is_unmapped, mapping_quality,
reference_name, query_alignment_sequence, query_alignment_qualities, reference_start and
cigartuples (main.py:165-173), with pysam's semantics (see basecount_amd/bam.py).
"""
from array import array

from basecount_amd.bam import BamFile

_verbosity = 3


def set_verbosity(v):
    global _verbosity
    old = _verbosity
    _verbosity = v
    return old


class AlignedSegment:
    __slots__ = ("_f", "_i")

    def __init__(self, f, i):
        self._f = f
        self._i = i

    @property
    def is_unmapped(self):
        return bool(int(self._f.flag[self._i]) & 4)

    @property
    def mapping_quality(self):
        return int(self._f.mapq[self._i])

    @property
    def reference_name(self):
        t = int(self._f.tid[self._i])
        return self._f.references[t] if 0 <= t < len(self._f.references) else None

    @property
    def reference_start(self):
        return int(self._f.pos[self._i])

    @property
    def cigartuples(self):
        return self._f.cigartuples(self._i)

    @property
    def query_alignment_sequence(self):
        if int(self._f.rec_err[self._i]) & 8:
            raise ValueError("Invalid clipping in CIGAR string")
        return self._f.query_alignment_sequence(self._i)

    @property
    def query_alignment_qualities(self):
        if int(self._f.rec_err[self._i]) & 8:
            raise ValueError("Invalid clipping in CIGAR string")
        q = self._f.query_alignment_qualities(self._i)
        return None if q is None else array("B", q.tobytes())


class AlignmentFile:
    def __init__(self, path, mode="rb"):
        self._f = BamFile(path)
        self.references = self._f.references
        self.lengths = self._f.lengths

    def fetch(self, contig=None, until_eof=False):
        for i in range(self._f.n_records):
            yield AlignedSegment(self._f, i)

    def close(self):
        self._f.close()
