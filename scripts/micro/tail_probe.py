"""k_tail alone on C4's contig (its kernel 2 outputs in place), with the 98 amplicon windows, with
none (the summary fold only) and with the windows but no summary tail: device time per launch
(hipEvents around 50 back-to-back launches).  python scripts/micro/tail_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402

from basecount_amd import device as D  # noqa: E402
from basecount_amd import synth  # noqa: E402
from basecount_amd.bam import seq_to_event  # noqa: E402
from basecount_amd.main import norm_factors  # noqa: E402
from basecount_amd.scheme import load_scheme  # noqa: E402
import tempfile  # noqa: E402

ctx = D.Context(0)
rs = synth.make_config("c3")
b = synth.batch_arrays(rs, 0, 0)
L, k = rs.lengths[0], 5
nf, nf2 = norm_factors(k)
r = D.DeviceReads(ctx, dict(b, qual=None, seq_event=seq_to_event(b["seq"])))
with tempfile.NamedTemporaryFile("w", suffix=".bed", delete=False) as fh:
    fh.write(synth.artic_bed())
tiles = [(w["inside_start"], w["inside_end"]) for _, _, w in load_scheme(fh.name)]
print("window lengths", min(b - a + 1 for a, b in tiles), max(b - a + 1 for a, b in tiles))
lo = np.array([t[0] for t in tiles], np.int64)
hi = np.array([t[1] for t in tiles], np.int64)
counts, cov, ent, sec = ctx.alloc(4 * k * L), ctx.alloc(4 * L), ctx.alloc(8 * L), ctx.alloc(8 * L)
work, dout = ctx.alloc(D.summary_work_bytes(L)), ctx.alloc(32)
dlo, dhi, damp = ctx.alloc(lo.nbytes).upload(lo), ctx.alloc(hi.nbytes).upload(hi), ctx.alloc(48 * len(tiles) + 128)
for nt in (len(tiles), 0, 1, 10):
    ctx.timing(True)
    for _ in range(30):
        ctx.pileup_summary_amplicons(r, L, 0, k, nf, nf2, counts.ptr, cov.ptr, ent.ptr, sec.ptr, work.ptr, dout.ptr,
                                     dlo.ptr, dhi.ptr, nt, damp.ptr)
    rep = ctx.timing_report()
    ctx.timing(False)
    print(nt, "windows:", {n: round(v[1], 2) for n, v in rep.items()}, flush=True)
    if nt and os.environ.get("TAIL_TRACE"):  # (-DBC_TAIL_TRACE build) block 1's phase stamps
        st = damp.download(np.float64, 6 * nt + 4)[6 * nt:]
        print("  stamps (cycles from phase 0):", [int(x - st[0]) for x in st], flush=True)
ctx.timing(True)
for _ in range(30):
    ctx.amplicons(cov.ptr, ent.ptr, sec.ptr, L, dlo.ptr, dhi.ptr, len(tiles), damp.ptr)
rep = ctx.timing_report()
ctx.timing(False)
print("k_amplicon alone:", {n: round(v[1], 2) for n, v in rep.items()}, flush=True)
