import os, sys
sys.path[:0] = ['.', 'oracle', 'tests']
import numpy as np
import oracle as O
from basecount_amd import device as D
from test_gpu_parity import random_batch, gpu_count
ctx = D.Context(0)
rng = np.random.default_rng(6)
b = random_batch(rng, 1_000_000, 2000)
exp, _ = O.bcount(1_000_000, 0, b)
for ab in ("0", "32"):
    os.environ["BC_ABLATE"] = ab
    got, bad = gpu_count(ctx, b, 1_000_000, 0, 5)
    e = exp[:, :5].T.astype(np.int32)
    d = np.nonzero((got != e).any(0))[0]
    print("ablate", ab, "bad", bad, "mismatching positions", d.size, d[:10], "tiles", np.unique(d // 64)[:10])
    if d.size:
        p = d[0]
        print(" got", got[:, p], "exp", e[:, p])
        t = p // 64
        sel = np.nonzero((b["pos"] < (t + 1) * 64) & (b["pos"] > t * 64 - 300))[0]
        print(" reads near tile", sel[:10], b["pos"][sel][:10], b["seq_nib"][sel][:10])
