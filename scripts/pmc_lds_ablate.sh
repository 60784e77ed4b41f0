#!/bin/bash
# Diagnostic: LDS counters and k_rc's duration under BC_ABLATE settings (DIAG build in
# scripts/tmp/libdiag.so); the in-tree library is restored at the end.
#   ABL="0 65536 16384 4" CONFIG=c3 bash scripts/pmc_lds_ablate.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG="${CONFIG:-c3}"; OUT=gpurun_out/pmc_lds; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=basecount_amd/libbasecount_hip.so
cp "$LIB" /tmp/lib_orig.so && cp scripts/tmp/libdiag.so "$LIB"
for a in $ABL; do
  BC_ABLATE=$a timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $OUT/a$a -o run -- python bench.py --config $CONFIG --allow-diag --no-cpu-baseline --no-extras --no-e2e --launch eager --lean --steps 20 --warmup 2 > $OUT/a$a.log 2>&1
  rc=$?; echo "ablate $a rc=$rc"; case $rc in 124|134|137|139) cp /tmp/lib_orig.so "$LIB"; exit $rc;; esac
done
cp /tmp/lib_orig.so "$LIB"
