#!/bin/bash
# Fold check: summary parity tests, C5 configs, the C5 kernel profile (one stream) and the C5 step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() {
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step r5f_parity 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "summary or fold or ctx_wait"
step r5f_configs 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py -k "c5"
step r5f_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5_f -o run -- \
    python bench.py --config c5 --no-cpu-baseline --no-extras --no-e2e --lean --launch eager --steps 5 --warmup 1 --streams 1
step r5f_c5 300 python bench.py --config c5 --no-cpu-baseline --no-extras --no-e2e --steps 10 --warmup 2
echo ALLDONE
