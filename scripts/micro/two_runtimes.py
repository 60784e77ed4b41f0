"""Probe: can torch's bundled HIP runtime and libbasecount_hip's (/opt/rocm) coexist in one process?"""
import sys
order = sys.argv[1]
import numpy as np
if order == "torch_first":
    import torch
    x = torch.ones(4, device="cuda"); torch.cuda.synchronize(); print("torch ok", float(x.sum()))
from basecount_amd import device as D
c = D.Context(0)
b = c.alloc(64); b.upload(np.arange(16, dtype=np.int32)); print("bc ok", b.download(np.int32, 16).sum())
if order == "bc_first":
    import torch
    x = torch.ones(4, device="cuda"); torch.cuda.synchronize(); print("torch ok", float(x.sum()))
