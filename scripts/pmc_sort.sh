#!/bin/bash
# PMC passes over the device sort of C3's reads in random order (scripts/micro/sort_ab.py), one
# counter group per run, --pmc with kernel-trace only:  bash scripts/pmc_sort.sh
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${OUT:-pmc_sort}; mkdir -p $OUT
root=$PWD
cd /tmp && export TMPDIR=/tmp
sets=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
      "FETCH_SIZE" "WRITE_SIZE")
for i in 1 2 3 4; do
  set=${sets[$((i-1))]}
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $root/$OUT/p$i -o run -- \
    python $root/scripts/micro/sort_ab.py 5 > $root/$OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
