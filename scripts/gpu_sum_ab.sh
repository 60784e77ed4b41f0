#!/bin/bash
# Summary-only change: the summary parity tests on the in-tree library, then C5 A/B against OLD
# (default scripts/tmp/lib_head.so), alternating, REPS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "summary or fold" > gpurun_out/sumab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/sumab_tests.log; [ $rc -eq 0 ] || exit $rc
cp basecount_amd/libbasecount_hip.so /tmp/lib_new.so
LIBS="/tmp/lib_new.so ${OLD:-scripts/tmp/lib_head.so}" CONFIG=c5 REPS=${REPS:-2} STEPS=10 bash scripts/ab_libs.sh
