#!/bin/bash
# k_rc / summary-only GPU check: parity tests, then the A/B and phase traces (exp_rc_phases.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 600 \
  --timeout-method thread -k "rc or kernel1 or fused or full_size or index or summary or c5_summary_only" > gpurun_out/t3.log 2>&1
rc=$?; tail -4 gpurun_out/t3.log; [ $rc -eq 0 ] || exit $rc
LIBS="$LIBS" REPS=2 bash scripts/exp_rc_phases.sh
