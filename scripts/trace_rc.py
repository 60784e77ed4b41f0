"""Summarize a k_rc BC_TRACE dump (diagnostic, -DBC_PHASE_TRACE build): per wave, s_memtime
cycles spent in each chunk phase, summed over its chunks.
    BC_TRACE=gpurun_out/rc.bin python bench.py --config c3 ...; python scripts/trace_rc.py gpurun_out/rc.bin"""
import sys
import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4, 7).astype(np.float64)
names = ["setup", "block_reduce", "records+stage wait", "expansion", "sum (w0-2) / flush (w3)",
         "counts+complex+end", "(unused)"]
tot = t.sum(axis=2)
print(f"blocks {t.shape[0]}; per-wave total cycles median {np.median(tot):.0f}")
for w in range(4):
    share = t[:, w, :].sum(axis=0) / t[:, w, :].sum()
    print(f"wave {w}: " + "  ".join(f"{n} {100 * s:.1f}%" for n, s in zip(names, share) if s > 0))
# absolute: median per-wave cycles of each phase, summed over the wave's chunks
med = np.median(t, axis=0)
for w in range(4):
    print(f"wave {w} cycles: " + "  ".join(f"{n} {m:.0f}" for n, m in zip(names, med[w]) if m > 0))
