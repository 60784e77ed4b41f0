#!/bin/bash
# A/B timing of bench.py argument variants in ONE GPU session:
#   VARIANTS="--summary-path=fused --summary-path=separate" CONFIG=c5 REPS=2 STEPS=10 bash scripts/ab_args.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG="${CONFIG:-c2}"; REPS="${REPS:-3}"; STEPS="${STEPS:-200}"
for rep in $(seq "$REPS"); do
  for v in $VARIANTS; do
    out=$(timeout -k 10 300 python bench.py --config "$CONFIG" --no-cpu-baseline --no-extras --no-e2e --steps "$STEPS" --warmup 2 ${v//,/ }) || { echo "FAILED $v"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '$CONFIG', round(d['ms_per_step']*1e3,2), 'us/step', {k: round(x,2) for k,x in d['kernel_us'].items()}, 'parity', d['parity_vs_oracle'])"
  done
done
