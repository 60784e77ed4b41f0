"""C3 sorted by start but with each read's sequence left where the unsorted batch had it (the
fields permuted, the sequence buffer not): k_rc's gather staging, against the same reads with a
contiguous sequence.  Graph-replayed bc_pileup steps, and parity with the oracle."""
import json
import os
import sys

import numpy as np

_R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(_R, "oracle"), _R]
import oracle as O  # noqa: E402
from basecount_amd import device as D, synth  # noqa: E402
from basecount_amd.bam import seq_to_event  # noqa: E402
from basecount_amd.main import norm_factors  # noqa: E402

ctx = D.Context(0)
rs = synth.make_config("c3", unsorted=True)
b = synth.batch_arrays(rs, 0, 0)
L, k = rs.lengths[0], 5
nf, nf2 = norm_factors(k)
o = np.argsort(b["pos"], kind="stable")
bs = dict(b, pos=b["pos"][o], cig_beg=b["cig_beg"][o], cig_n=b["cig_n"][o], seq_nib=b["seq_nib"][o])
exp, _ = O.bcount(L, 0, b, nthreads=8)
out = {}
bufs = [ctx.alloc(n) for n in (4 * k * L, 4 * L, 8 * k * L, 8 * L, 8 * L)]
for name, bb in (("gather", bs), ("contiguous", synth.batch_arrays(synth.make_config("c3"), 0, 0))):
    r = D.DeviceReads(ctx, dict(bb, qual=None, seq_event=seq_to_event(bb["seq"])))
    assert r.r.sorted == 1
    step = lambda: ctx.pileup(r, L, 0, k, nf, nf2, *[x.ptr for x in bufs])  # noqa: E731
    for _ in range(3):
        step()
    g = ctx.capture(lambda: [step() for _ in range(20)])
    g.launch()
    ctx.sync()
    ctx.event_record(2)
    g.launch()
    ctx.event_record(3)
    ctx.sync()
    us = ctx.event_elapsed_ms(2, 3) * 1e3 / 20
    del g
    ctx.timing(True)
    for _ in range(20):
        step()
    rep = ctx.timing_report()
    ctx.timing(False)
    got = bufs[0].download(np.int32, k * L).reshape(k, L)
    e = exp if name == "gather" else O.bcount(L, 0, bb, nthreads=8)[0]
    out[name] = {"step_us": us, "k_rc_us": rep["rc"][1], "parity": bool(np.array_equal(got, e[:, :k].T.astype(np.int32)))}
    r.free()
print(json.dumps(out, indent=1))
