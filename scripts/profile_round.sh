#!/bin/bash
# The round's profiles in one GPU session: rocprofv3 kernel traces (--kernel-trace --stats) of
# the bench per config (CFGS, default c2 c3 c3q20 c4 c5), then separate PMC passes (instruction and
# wait counters, LDS, HBM bytes: FETCH_SIZE, WRITE_SIZE) for every config.  Stops at the first
# fault / abort / timeout.  Then, on the CPU:
#   for c in c2 c3 c3q20 c4 c5 c3unsorted; do cp gpurun_out/prof_$c/run_kernel_stats.csv profiles/r0N_${c}_kernel_stats.csv; done
#   python scripts/pmc_json.py profiles/r0N_pmc.json profiles/kernel1_pmc.json c2=gpurun_out/pmc_c2:k_pileup:pileup:<copies> ...
# (the copies of each config: batch_copies in gpurun_out/prof_<c>.log)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for c in ${CFGS:-c2 c3 c3q20 c4 c5}; do
  steps=200; extra=""; cfg=$c
  [ "$c" = c5 ] && steps=5 && extra="--streams 1"  # c5: launches serialized, so their durations add up
  [ "$c" = c3q20 ] && cfg=c3 && extra="--mbq 20"   # C3 with the quality test (QUAL bytes read)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o run -- \
    python bench.py --config $cfg --no-cpu-baseline --no-extras --no-e2e --lean --launch eager --steps $steps --warmup 2 $extra \
    > gpurun_out/prof_$c.log 2>&1
  rc=$?; echo "trace $c rc=$rc"; fatal $rc && exit $rc
  pargs="--config $cfg"; [ "$c" = c3q20 ] && pargs="$pargs --mbq 20"; [ "$c" = c5 ] && pargs="$pargs --steps 5 --streams 1"
  PASSES="${PASSES:-1 2 3 4 5}" BENCH_ARGS="$pargs" OUT=pmc_$c bash scripts/pmc.sh
  rc=$?; fatal $rc && exit $rc
done
# the unsorted C3 leg (bench.run_unsorted: the device sort, then k_rc on the sorted view)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3unsorted -o run -- \
  python scripts/prof_unsorted.py > gpurun_out/prof_c3unsorted.log 2>&1
rc=$?; echo "trace c3unsorted rc=$rc"; fatal $rc && exit $rc
echo PROFILES_DONE
