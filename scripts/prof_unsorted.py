"""The bench's unsorted-C3 leg alone (bench.run_unsorted: the same batches, copies and graphs), its
result line printed, for a rocprofv3 kernel trace whose per-kernel averages match the leg's own
figures:
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_uns -o run -- python scripts/prof_unsorted.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from basecount_amd.main import context  # noqa: E402

ctx = context()
print(json.dumps(bench.compact(bench.run_unsorted(ctx, None))), flush=True)
