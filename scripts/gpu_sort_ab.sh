#!/bin/bash
# A/B of the device sort (bucketed vs the counting sort with global atomics) in one gpurun call:
# the sort tests, then the sort's device time per variant, alternating, then a kernel trace.
set -e -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_configs.py -k "sort or unsorted" > gpurun_out/sortab_tests.log 2>&1
for i in 1 2; do
    timeout -k 10 120 python -u scripts/micro/sort_ab.py 20 >> gpurun_out/sortab.log 2>&1
    BC_SORT_BKT=0 timeout -k 10 120 python -u scripts/micro/sort_ab.py 20 >> gpurun_out/sortab.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sort" -o run -- \
    python -u "$GRAFT_REPO_ROOT/scripts/micro/sort_ab.py" 20 >> "$GRAFT_REPO_ROOT/gpurun_out/sortab.log" 2>&1
