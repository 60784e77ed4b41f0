"""The streaming BAM decoder (bcio_stream_*, bam.BamStream) on the CPU: batches reproduce the
whole-file decode record for record, truncated files fail like the whole-file decoder, and the
peak memory of a streamed pass does not grow with the file (--chunk-size must
bound memory, /root/reference/basecount/main.py:142-162)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from basecount_amd import synth
from basecount_amd.bam import BamFile, BamStream

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
REPO = os.path.dirname(HERE)

FIELDS = ("tid", "pos", "flag", "mapq", "l_seq", "qstart", "qend", "rec_err", "ref_span")


@pytest.mark.parametrize("bam", ["c1.bam", "mixed.bam", "edge.bam", "err_order.bam"])
@pytest.mark.parametrize("batch", [1, 3, 250, 10 ** 9])
def test_stream_batches_equal_whole_file(bam, batch):
    path = os.path.join(GOLDEN, bam)
    with BamFile(path) as f:
        whole = {k: getattr(f, k).copy() for k in FIELDS}
        cig = [f.cigartuples(i) for i in range(f.n_records)]
        seqs = [f.query_alignment_sequence(i) for i in range(f.n_records)]
        refs, lens, n = f.references, f.lengths, f.n_records
    got = {k: [] for k in FIELDS}
    gcig, gseq = [], []
    with BamStream(path) as s:
        assert s.references == refs and s.lengths == lens
        seen = 0
        for b in s.batches(batch):
            assert b.first_record == seen and 0 < b.n_records <= batch
            seen += b.n_records
            for k in FIELDS:
                got[k].append(getattr(b, k).copy())
            gcig += [b.cigartuples(i) for i in range(b.n_records)]
            gseq += [b.query_alignment_sequence(i) for i in range(b.n_records)]
    assert seen == n
    for k in FIELDS:
        assert np.array_equal(np.concatenate(got[k]), whole[k]), k
    assert gcig == cig and gseq == seqs


def test_stream_selection_ordinals_continue_across_batches():
    """Per batch, bcio_select's ordinals count from the batch start: offset by the accepted reads
    before it, they are the whole file's (the reference's chunk positions, main.py:142)."""
    path = os.path.join(GOLDEN, "mixed.bam")
    with BamFile(path) as f:
        sel = f.select(30, [True])
        whole = (sel.ordinal.copy(), sel.pos.copy(), f.n_records)
    ords, pos, base = [], [], 0
    with BamStream(path) as s:
        for b in s.batches(333):
            sb = b.select(30, [True])
            ords.append(sb.ordinal + base)
            pos.append(sb.pos.copy())
            base += sb.n_accepted
    assert np.array_equal(np.concatenate(ords), whole[0])
    assert np.array_equal(np.concatenate(pos), whole[1])


def test_stream_truncated_file_fails(tmp_path):
    src = open(os.path.join(GOLDEN, "c1.bam"), "rb").read()
    for cut in (10, 30, len(src) // 2, len(src) - 5):
        p = tmp_path / f"cut{cut}.bam"
        p.write_bytes(src[:cut])
        with pytest.raises(ValueError):
            with BamStream(str(p)) as s:
                for _ in s.batches(100):
                    pass


# peak resident set of the child's own address space (VmHWM: ru_maxrss would carry over the
# parent's high-water mark across fork + exec)
_RSS = """
import sys
sys.path.insert(0, {repo!r})
from basecount_amd.bam import BamStream, BamFile
n = 0
if sys.argv[2] == "stream":
    with BamStream(sys.argv[1]) as s:
        for b in s.batches(int(sys.argv[3])):
            sel = b.select(0, [True] * len(s.references))
            n += b.n_records
else:
    with BamFile(sys.argv[1]) as f:
        sel = f.select(0, [True] * len(f.references))
        n = f.n_records
hwm = [ln for ln in open("/proc/self/status") if ln.startswith("VmHWM:")][0].split()[1]
print(n, hwm)
"""


def _peak_kb(bam, mode, batch=0):
    out = subprocess.run([sys.executable, "-c", _RSS.format(repo=REPO), bam, mode, str(batch)],
                         capture_output=True, timeout=600, check=True).stdout.decode().split()
    return int(out[0]), int(out[1])


def test_stream_peak_memory_independent_of_read_count(tmp_path):
    """At a fixed batch size, streaming 4x the reads keeps the same peak RSS; decoding the whole
    file grows with it."""
    paths = {}
    for n in (100_000, 400_000):
        rs = synth.make_reads([("chrS", 2_000_000)], n, True, 17)
        paths[n] = str(tmp_path / f"s{n}.bam")
        synth.write_bam(rs, paths[n])
        del rs
    n1, s_small = _peak_kb(paths[100_000], "stream", 20_000)
    n2, s_big = _peak_kb(paths[400_000], "stream", 20_000)
    assert (n1, n2) == (100_000, 400_000)
    _, w_small = _peak_kb(paths[100_000], "whole")
    _, w_big = _peak_kb(paths[400_000], "whole")
    # the whole-file decode holds ~400 B per read more; the stream does not
    assert w_big - w_small > 60_000, (w_small, w_big)
    assert s_big - s_small < 0.25 * (w_big - w_small), (s_small, s_big, w_small, w_big)
