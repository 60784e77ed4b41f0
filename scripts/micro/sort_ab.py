"""bc_reads_sort on C3's reads in random order: the sort's device time (library timing, mean of
REPS calls) and the sorted copy's counts against the unsorted batch's.  Run once per variant
(BC_SORT_BKT=0 selects the counting sort with global atomics):
    python scripts/micro/sort_ab.py [reps] [unsorted|sorted]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402

from basecount_amd import device as D  # noqa: E402
from basecount_amd import synth  # noqa: E402
from basecount_amd.bam import seq_to_event  # noqa: E402
from basecount_amd.main import norm_factors  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
order = sys.argv[2] if len(sys.argv) > 2 else "unsorted"  # "sorted": C3's batch in start order
ctx = D.Context(0)
rs = synth.make_config("c3", unsorted=order != "sorted")
b = synth.batch_arrays(rs, 0, 0)
L, k = rs.lengths[0], 5
nf, nf2 = norm_factors(k)
reads = D.DeviceReads(ctx, dict(b, qual=None, seq_event=seq_to_event(b["seq"])))
counts = ctx.alloc(4 * k * L)
nb = ctx.sort_bytes(reads)
mem = ctx.alloc(nb)
srt = ctx.sort(reads, mem.ptr, nb)
ctx.timing(True)
for _ in range(reps):
    srt = ctx.sort(reads, mem.ptr, nb)
sort_us = ctx.timing_report()["sort"][1]
ctx.timing(False)
pos = np.zeros(srt.n_reads, np.int32)
D.check(D.lib().bc_memcpy_d2h(ctx.h, pos.ctypes.data, srt.pos, pos.nbytes))
ctx.sync()
sorted_ok = bool(np.array_equal(pos, np.sort(b["pos"])))
ref = ctx.alloc(4 * k * L)
ref.zero()
ctx.count(reads, L, 0, k, ref.ptr)
counts.zero()
ctx.count(srt, L, 0, k, counts.ptr)
same = bool(np.array_equal(ref.download(np.int32, k * L), counts.download(np.int32, k * L)))
print(f"variant={os.environ.get('BC_SORT_BKT', 'default')} order={order} sort_us={sort_us:.1f} sorted={sorted_ok} counts_equal={same}",
      flush=True)
