import sys, numpy as np
t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 7).astype(np.float64)
names = ["decode", "reduce", "stage+rec", "expand", "accum", "flush+end"]
tot = t[:, :6].sum(axis=1)
print("waves", len(t), "median total cycles", np.median(tot))
for i, n in enumerate(names):
    print(f"{n:10s} median {np.median(t[:, i]):9.0f}  mean {np.mean(t[:, i]):9.0f}  frac {np.sum(t[:, i]) / np.sum(tot):.3f}")
