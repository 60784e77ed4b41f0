"""bench.run_unsorted alone (C3 in random order: event-parallel, sort + sorted path, in place)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from basecount_amd import device as D  # noqa: E402

print(json.dumps(bench.run_unsorted(D.Context(0), None), indent=1))
