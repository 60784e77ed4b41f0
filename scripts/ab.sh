#!/bin/bash
# A/B timing of environment variants in ONE GPU session (boxes differ by up to 25 %):
#   VARIANTS="BC_ABLATE=0 BC_ABLATE=256" CONFIG=c2 REPS=3 bash scripts/ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG="${CONFIG:-c2}"; REPS="${REPS:-3}"; STEPS="${STEPS:-200}"
for rep in $(seq "$REPS"); do
  for v in $VARIANTS; do
    out=$(env ${v//,/ } timeout -k 10 300 python bench.py --config "$CONFIG" --no-cpu-baseline --steps "$STEPS" --warmup 20) || { echo "FAILED $v"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['device_us_per_step'],2), 'us', d['kernel_us'], 'parity', d['parity_vs_oracle'])"
  done
done
