#!/bin/bash
# Round 5, first session: the read-parallel summary (bc_sum.hip) parity tests, the C5 A/B against
# the per-tile sweep (lib_sweep.so, -DBC_SUM_SWEEP), and the new C4 bench leg.  Stops at the first
# failure; every GPU step has its own time limit.
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
step r5a_parity 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "summary or fold or ctx_wait"
step r5a_configs 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py \
  -k "c5_summary_only or c5_cli"
cp basecount_amd/libbasecount_hip.so scripts/tmp/lib_new.so
step r5a_ab_c5 600 env LIBS="scripts/tmp/lib_new.so scripts/tmp/lib_sweep.so" CONFIG=c5 REPS=2 STEPS=10 \
  bash scripts/ab_libs.sh
step r5a_c4 600 python bench.py --config c4 --no-cpu-baseline --no-extras --no-e2e --steps 50 --warmup 5
echo ALLDONE
