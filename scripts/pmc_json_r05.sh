#!/bin/bash
# profiles/r05_pmc.json + profiles/kernel1_pmc.json from this round's PMC passes (gpurun_out/pmc_*)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python scripts/pmc_json.py profiles/r05_pmc.json profiles/kernel1_pmc.json \
  c2=gpurun_out/pmc_c2:k_pileup:pileup:1 c3=gpurun_out/pmc_c3:k_rc:rc:3 c3_q20=gpurun_out/pmc_c3q20:k_rc:rc:3:1:20 \
  c4=gpurun_out/pmc_c4:k_rc:rc:3 c4_amplicon=gpurun_out/pmc_c4:k_amplicon:amplicons:3 \
  c5=gpurun_out/pmc_c5:k_sum_reads+k_sum_exact+k_sum_buffers:solo_sum:1:24
