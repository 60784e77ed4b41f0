#!/bin/bash
# A/B timing of BC_ABLATE settings with a diagnostic build (scripts/tmp/libdiag.so, make DIAG=1)
# in ONE GPU session; the in-tree library is restored at the end.  Diagnostic numbers only.
#   ABL="0 16384 32768" CONFIG=c3 REPS=2 bash scripts/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG="${CONFIG:-c2}"; REPS="${REPS:-2}"; STEPS="${STEPS:-200}"
LIB=basecount_amd/libbasecount_hip.so
cp "$LIB" /tmp/lib_orig.so
cp scripts/tmp/libdiag.so "$LIB"
for rep in $(seq "$REPS"); do
  for a in $ABL; do
    # (exit 3 = parity false: expected when an ablation skips work; anything else stops the A/B)
    out=$(BC_ABLATE=$a timeout -k 10 300 python bench.py --config "$CONFIG" --allow-diag --no-cpu-baseline --no-extras --no-e2e --steps "$STEPS" --warmup 5 ${BENCH_ARGS}); rc=$?
    [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "FAILED $a rc=$rc"; cp /tmp/lib_orig.so "$LIB"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ablate=$a', '$CONFIG', round(d['ms_per_step']*1e3,2), 'us/step', {k: round(x,2) for k,x in d['kernel_us'].items()})"
  done
done
cp /tmp/lib_orig.so "$LIB"
