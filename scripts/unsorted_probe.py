"""The unsorted-C3 measurement of bench.py alone (bench.run_unsorted), for kernel traces:
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_u -o run -- python3 scripts/unsorted_probe.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from basecount_amd.main import context  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.run_unsorted(context(), None, reps=int(sys.argv[1]) if len(sys.argv) > 1 else 10)))
