#!/bin/bash
# One GPU session: smoke -> gpu tests -> bench -> rocprof kernel trace.  Stops at the first
# fault / abort / timeout (exit 124, 134, 137, 139) so a broken kernel never runs twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-smoke tests bench prof}"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 ${PYTEST_ARGS} ;;
    bench) run bench 600 python bench.py ${BENCH_ARGS} ;;
    bench3) run bench3 600 python bench.py --config c3 --no-cpu-baseline --no-extras ${BENCH_ARGS} ;;
    bench5) run bench5 600 python bench.py --config c5 --no-cpu-baseline --no-extras --steps 10 --warmup 2 ${BENCH_ARGS} ;;
    e2e)   run e2e 900 bash -c "python scripts/e2e.py --config c2 && python scripts/e2e.py --config c3 && python scripts/e2e.py --config c5 --summarise" ;;
    prof)  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
           run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --no-cpu-baseline --no-extras --no-e2e --launch eager --steps 200 ${BENCH_ARGS} ;;
    prof5) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
           run prof5 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o run -- python bench.py --no-cpu-baseline --no-extras --launch eager --steps 5 --warmup 1 --config c5 ${BENCH_ARGS} ;;
    prof3) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
           run prof3 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python bench.py --no-cpu-baseline --no-extras --launch eager --steps 200 --config c3 ${BENCH_ARGS} ;;
  esac
done
echo ALLDONE
