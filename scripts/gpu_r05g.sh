#!/bin/bash
# fold A/B (microbenchmark), then the k_rc phase traces (single pass and indexed).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_fold_ab.sh || exit 1
bash scripts/exp_rc_phases.sh
