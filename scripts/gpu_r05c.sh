#!/bin/bash
# Round 5, third session: the integer-run fold, scratch release, the chromosome-scale pileup test,
# the k_rc clean-up (rejected variants removed, gather staging only when reads fit their slots),
# and the N>1 headline (C5) rehearsed with two ranks on one GPU.
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
step r5c_parity 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "summary or fold or amplicon or 64bit or rc_ or gather or ctx_wait" tests/test_gpu_api.py tests/test_capi.py
step r5c_configs 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py \
  -k "c5 or c4"
step r5c_c5 600 python bench.py --config c5 --no-cpu-baseline --no-extras --no-e2e --steps 10 --warmup 2
step r5c_dist2 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_dist.py -k bench_gpus_2
echo ALLDONE
