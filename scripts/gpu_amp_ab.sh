#!/bin/bash
# k_amplicon change: amplicon parity tests and the C4 CLI configs, then C4 A/B against OLD
# (default scripts/tmp/lib_head.so), alternating, REPS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_configs.py -k "amplicon or summary or fold or c4 or c5" > gpurun_out/ampab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ampab_tests.log; [ $rc -eq 0 ] || exit $rc
cp basecount_amd/libbasecount_hip.so /tmp/lib_new.so
LIBS="/tmp/lib_new.so ${OLD:-scripts/tmp/lib_head.so}" CONFIG=c4 REPS=${REPS:-2} STEPS=50 bash scripts/ab_libs.sh
