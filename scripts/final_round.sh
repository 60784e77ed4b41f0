#!/bin/bash
# One GPU session at the end of a change: the A/B given in LIBS (optional), then smoke, the GPU
# suite, the default bench line and the profiles (kernel traces + PMC passes) of the in-tree
# library.  Stops at the first fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ -n "$LIBS" ]; then
  LIBS="$LIBS" CONFIG=${AB_CONFIG:-c3} REPS=${REPS:-3} bash scripts/ab_libs.sh > gpurun_out/ab_final.log 2>&1
  rc=$?; echo "ab rc=$rc"; tail -12 gpurun_out/ab_final.log | cut -c1-160; fatal $rc && exit $rc
fi
STEPS="smoke tests bench" bash scripts/gpu_round.sh || exit $?
grep -q "FATAL" gpurun_out/*.log 2>/dev/null && exit 1
CFGS="${CFGS:-c3 c2 c5}" bash scripts/profile_round.sh
