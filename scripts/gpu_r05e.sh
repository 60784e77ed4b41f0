#!/bin/bash
# Fold rework check: summary parity tests, C5 configs, then the C5 kernel profile (cur vs OLD).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step r5e_parity 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "summary or fold or ctx_wait"
step r5e_configs 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py -k "c5"
bash scripts/gpu_r05d.sh
