#!/bin/bash
# PMC passes over the C2 bench (each pass its own run, --pmc with kernel-trace only)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py --no-cpu-baseline --steps 20 --warmup 2 ${BENCH_ARGS} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
done
