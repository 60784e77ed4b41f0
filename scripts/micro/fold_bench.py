"""Microbenchmark of the summary fold (k_sum_final via bc_summary_fold) on crafted per-buffer
partials: m buffers, a fraction `frac` of them fractional, the rest integers, against a Python
sequential float64 sum (the fold's definition).  Prints us per launch per case.
    python scripts/micro/fold_bench.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from basecount_amd import device as D  # noqa: E402

ctx = D.Context(0)
rng = np.random.default_rng(5)
for m, frac in ((30390, 0.0), (30390, 0.045), (30390, 1.0), (5701, 0.67), (30390 * 4, 0.045)):
    L = m * 8192
    ent = np.where(rng.random(m) < frac, rng.random(m) * 8192, rng.integers(0, 8193, m).astype(np.float64))
    cov = rng.integers(0, 1000, m).astype(np.int64)
    nz = rng.integers(0, 1000, m).astype(np.int64)
    wb = D.summary_work_bytes(L)
    host = np.zeros(wb, np.uint8)
    # layout (bc_kernels.hip summary_parts): 16 B header, ent[nc], cov[nc], nz[nc], quarters
    host[16:16 + 8 * m] = ent.view(np.uint8)
    host[16 + 8 * m:16 + 16 * m] = cov.view(np.uint8)
    host[16 + 16 * m:16 + 24 * m] = nz.view(np.uint8)
    work = ctx.alloc(wb).upload(host)
    out = ctx.alloc(32)
    ctx.summary_fold([L], [work.ptr], [out.ptr])
    ctx.sync()
    reps = 20
    ctx.event_record(0)
    for _ in range(reps):
        ctx.summary_fold([L], [work.ptr], [out.ptr])
    ctx.event_record(1)
    us = ctx.event_elapsed_ms(0, 1) * 1e3 / reps
    s = 0.0
    for v in ent.tolist():
        s += v
    got = out.download(np.float64, 4)
    ok = got[1] == s / L and got[3] == float(cov.sum())
    hdr = work.download(np.uint32, 4)  # a BC_FOLD_TRACE build leaves thread 0's phase cycles here
    tr = ""
    if hdr[1] or hdr[2]:
        tr = (f"  [trace: scan {hdr[1] * 64 / 2.4e3:.1f} us, chain {hdr[2] * 64 / 2.4e3:.1f} us, "
              f"check {(hdr[3] & 0xFFFFFF) * 64 / 2.4e3:.1f} us, redos {hdr[3] >> 24}]")
    print(f"m={m:7d} frac={frac:5.3f}: {us:8.1f} us per fold, exact={ok}{tr}", flush=True)
