#!/bin/bash
# One GPU session for a k_rc change: the k_rc / kernel-1 parity tests with the in-tree library,
# then the A/B of LIBS at C3 (scripts/ab_libs.sh).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${TESTS_K:-rc or kernel1 or fused or full_size or sort or index}" > gpurun_out/t_rc.log 2>&1
rc=$?; tail -3 gpurun_out/t_rc.log; [ $rc -eq 0 ] || exit $rc
[ -n "$LIBS" ] || exit 0
LIBS="$LIBS" CONFIG=${CONFIG:-c3} REPS=${REPS:-2} bash scripts/ab_libs.sh > gpurun_out/ab_c3.log 2>&1
rc=$?; cat gpurun_out/ab_c3.log; exit $rc
