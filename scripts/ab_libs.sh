#!/bin/bash
# A/B timing of alternative builds of libbasecount_hip.so in ONE GPU session (boxes differ by up
# to ~10 %): each variant file is copied over the in-tree library before its runs, the original
# is restored at the end.
#   LIBS="scripts/tmp/libA.so scripts/tmp/libB.so" CONFIG=c3 REPS=3 bash scripts/ab_libs.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG="${CONFIG:-c2}"; REPS="${REPS:-3}"; STEPS="${STEPS:-200}"
LIB=basecount_amd/libbasecount_hip.so
cp "$LIB" /tmp/lib_orig.so
for rep in $(seq "$REPS"); do
  for v in $LIBS; do
    cp "$v" "$LIB"
    out=$(timeout -k 10 300 python bench.py --config "$CONFIG" --no-cpu-baseline --no-extras --no-e2e --steps "$STEPS" --warmup 20 ${BENCH_ARGS}) || { echo "FAILED $v"; cp /tmp/lib_orig.so "$LIB"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $v)', '$CONFIG', round(d['ms_per_step']*1e3,2), 'us/step', {k: round(x,2) for k,x in d['kernel_us'].items()}, 'parity', d['parity_vs_oracle'])"
  done
done
cp /tmp/lib_orig.so "$LIB"
