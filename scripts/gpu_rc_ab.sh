#!/bin/bash
# k_rc change: the rc parity tests, then A/B at C3 (and C3 q20) of the in-tree library against
# OLD (default scripts/tmp/lib_rc_old.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "rc_ or kernel1 or 64bit or gather or full_size or device_sort or pileup_shapes" > gpurun_out/rcab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rcab_tests.log; [ $rc -eq 0 ] || exit $rc
cp basecount_amd/libbasecount_hip.so /tmp/lib_new.so
LIBS="/tmp/lib_new.so ${OLD:-scripts/tmp/lib_rc_old.so}" CONFIG=c3 REPS=${REPS:-3} bash scripts/ab_libs.sh || exit 1
LIBS="/tmp/lib_new.so ${OLD:-scripts/tmp/lib_rc_old.so}" CONFIG=c3 REPS=1 BENCH_ARGS="--mbq 20" bash scripts/ab_libs.sh
