#!/bin/bash
# Diagnostic: instruction counters of one config under BC_ABLATE settings, with the DIAG build
# (scripts/tmp/libdiag.so, make DIAG=1); the in-tree library is restored at the end.
#   ABL="0 4 2048" CONFIG=c3 KERNEL=k_rc bash scripts/pmc_ablate.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG="${CONFIG:-c3}"; OUT=gpurun_out/pmc_abl; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=basecount_amd/libbasecount_hip.so
cp "$LIB" /tmp/lib_orig.so && cp scripts/tmp/libdiag.so "$LIB"
for a in $ABL; do
  BC_ABLATE=$a timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/a$a -o run -- python bench.py --config $CONFIG --allow-diag --no-cpu-baseline --no-extras --no-e2e --launch eager --steps 20 --warmup 2 > $OUT/a$a.log 2>&1
  rc=$?; echo "ablate $a rc=$rc"; case $rc in 124|134|137|139) cp /tmp/lib_orig.so "$LIB"; exit $rc;; esac
done
cp /tmp/lib_orig.so "$LIB"
