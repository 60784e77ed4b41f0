#!/bin/bash
# One GPU session: A/B of LIBS at C3, then the k_rc phase traces (-DBC_PHASE_TRACE build in
# scripts/tmp/lib_trace.so) of the indexed and the CIGAR-decoding step.  Diagnostic only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=basecount_amd/libbasecount_hip.so
cp $LIB /tmp/lib_orig.so
if [ -n "$LIBS" ]; then
  LIBS="$LIBS" CONFIG=c3 REPS=${REPS:-2} bash scripts/ab_libs.sh > gpurun_out/ab_exp.log 2>&1 || { cat gpurun_out/ab_exp.log; exit 1; }
  cat gpurun_out/ab_exp.log
fi
cp scripts/tmp/lib_trace.so $LIB
for m in idx noidx; do
  extra="--read-runs off"; [ $m = idx ] && extra="--read-runs on"
  BC_TRACE=gpurun_out/rc_$m.bin timeout -k 10 300 python bench.py --config c3 --no-extras --no-e2e --no-cpu-baseline \
    --steps 20 --warmup 5 --launch eager --lean --allow-diag $extra > gpurun_out/tr_$m.log 2>&1
  rc=$?; echo "trace $m rc=$rc"; [ $rc -eq 0 ] || { cp /tmp/lib_orig.so $LIB; tail -5 gpurun_out/tr_$m.log; exit $rc; }
  python scripts/trace_rc.py gpurun_out/rc_$m.bin
done
cp /tmp/lib_orig.so $LIB
