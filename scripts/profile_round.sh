#!/bin/bash
# The round's profiles in one GPU session: rocprofv3 kernel traces (--kernel-trace --stats) of
# the bench for c2 / c3 / c5, then separate PMC passes (HBM bytes: FETCH_SIZE, WRITE_SIZE; and the
# instruction counters for c2 / c3).  Stops at the first fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for c in ${CFGS:-c2 c3 c5}; do
  steps=200; extra=""; [ "$c" = c5 ] && steps=5 && extra="--streams 1"  # c5: launches serialized, so their durations add up
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o run -- \
    python bench.py --config $c --no-cpu-baseline --no-extras --no-e2e --lean --launch eager --steps $steps --warmup 2 $extra \
    > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "trace $c rc=$rc"; fatal $rc && exit $rc
  passes="4 5"; [ "$c" != c5 ] && passes="1 2 3 4 5"
  PASSES="$passes" BENCH_ARGS="--config $c" OUT=pmc_$c bash scripts/pmc.sh
  rc=$?; fatal $rc && exit $rc
done
echo PROFILES_DONE
