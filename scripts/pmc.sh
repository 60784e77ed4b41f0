#!/bin/bash
# PMC passes over the bench (one counter group per run, --pmc with kernel-trace only).
#   PASSES="1 2 3" BENCH_ARGS="--config c3" OUT=pmc3 bash scripts/pmc.sh
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUT:-pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
sets=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
      "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
      "FETCH_SIZE" "WRITE_SIZE")
for i in ${PASSES:-1 2 3 4 5}; do
  set=${sets[$((i-1))]}
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python bench.py --no-cpu-baseline --no-extras --no-e2e --lean --launch eager --steps 20 --warmup 2 ${BENCH_ARGS} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done
