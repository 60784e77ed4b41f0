"""Summarize a BC_TRACE dump (diagnostic): per-wave phase stamps of one k_pileup launch.
    BC_TRACE=gpurun_out/trace.bin python bench.py --steps 30 --no-cpu-baseline; python scripts/trace_phases.py gpurun_out/trace.bin
Phases: 0 start, 1 range search shared, 2 first chunk walked, 3 second chunk walked, 4 wave partials
reduced, 5 counts written, 6 fp64 terms done, 7 tile done.  Units: us from the first wave's start."""
import sys
import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 12).astype(np.float64)
nw = int(sys.argv[2]) if len(sys.argv) > 2 else 8
valid = t[:, 0] > 0
t = t[valid]
t0 = t[:, 0].min()
us = (t - t0) / 100.0  # s_memrealtime: 100 MHz
us[t[:, :] == 0] = np.nan
names = ["start", "search", "chunk1", "chunk2", "reduce", "counts", "terms", "end", "probe1", "srchend", "probe2", "cigar1"]
print(f"waves {len(us)}; kernel span {np.nanmax(us):.2f} us")
for i, n in enumerate(names):
    col = us[:, i]
    if np.all(np.isnan(col)):
        continue
    print(f"{n:7s} min {np.nanmin(col):6.2f}  median {np.nanmedian(col):6.2f}  p90 {np.nanpercentile(col, 90):6.2f}  max {np.nanmax(col):6.2f}")
