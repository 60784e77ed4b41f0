#!/bin/bash
# A/B of the unsorted-C3 leg (bench.run_unsorted: sort + sorted path from the raw unsorted batch)
# over alternative builds of libbasecount_hip.so in ONE GPU session, alternating:
#   LIBS="scripts/tmp/libA.so scripts/tmp/libB.so" REPS=2 bash scripts/ab_unsorted.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPS="${REPS:-2}"
LIB=basecount_amd/libbasecount_hip.so
cp "$LIB" /tmp/lib_orig.so
for rep in $(seq "$REPS"); do
  for v in $LIBS; do
    cp "$v" "$LIB"
    out=$(timeout -k 10 300 python scripts/prof_unsorted.py | grep '^{') || { echo "FAILED $v"; cp /tmp/lib_orig.so "$LIB"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $v)', {k: d[k] for k in ('sort_us', 'unsorted_step_us', 'sorted_input_step_us', 'ratio_to_sorted_input', 'parity_vs_oracle')})"
  done
done
cp /tmp/lib_orig.so "$LIB"
