"""C3 unsorted: bc_reads_sort then the sorted path, 20 times (for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_uns -o run -- python scripts/prof_unsorted.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from basecount_amd import device as D  # noqa: E402
from basecount_amd import synth  # noqa: E402
from basecount_amd.bam import seq_to_event  # noqa: E402
from basecount_amd.main import norm_factors  # noqa: E402

ctx = D.Context(0)
rs = synth.make_config("c3", unsorted=True)
b = synth.batch_arrays(rs, 0, 0)
L, k = rs.lengths[0], 5
nf, nf2 = norm_factors(k)
reads = D.DeviceReads(ctx, dict(b, qual=None, seq_event=seq_to_event(b["seq"])))
counts, cov, pc = ctx.alloc(4 * k * L), ctx.alloc(4 * L), ctx.alloc(8 * k * L)
ent, sec = ctx.alloc(8 * L), ctx.alloc(8 * L)
nb = ctx.sort_bytes(reads)
mem = ctx.alloc(nb)
for _ in range(20):  # stream-ordered: the sort only enqueues
    srt = ctx.sort(reads, mem.ptr, nb, check_flags=False)
    ctx.pileup(srt, L, 0, k, nf, nf2, counts.ptr, cov.ptr, pc.ptr, ent.ptr, sec.ptr)
ctx.sync()
ctx.sort_check(reads, mem.ptr)
print("done")
