#!/bin/bash
# Round 5, second session: the amplicon medians (wave bitonic sort), C4 and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step r5b_parity 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "amplicon or summary_only_scratch"
step r5b_c4cli 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k c4
step r5b_bench 900 python bench.py
echo ALLDONE
