#!/bin/bash
# Round 5's closing GPU sessions on the final library, by STAGE:
#   A  the sort tests and A/B, the unsorted sort's kernel trace, then the profiles of c2 c3 c3q20
#   B  the profiles of c4 c5, then the default bench line
#   C  smoke, the whole GPU suite and the default bench line (with the PMC traffic of this library)
#   ALL  A + B's profiles + the PMC summaries (scripts/pmc_json_r05.sh) + C, in one session
# Every GPU step has its own time limit and the steps are chained: the first failure ends the call.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
case "${STAGE:?STAGE=A|B|C}" in
  A)
    bash scripts/gpu_sort_ab.sh
    CFGS="c2 c3 c3q20" bash scripts/profile_round.sh > gpurun_out/final_prof_a.log 2>&1
    grep -q PROFILES_DONE gpurun_out/final_prof_a.log
    ;;
  B)
    CFGS="c4 c5" bash scripts/profile_round.sh > gpurun_out/final_prof_b.log 2>&1
    grep -q PROFILES_DONE gpurun_out/final_prof_b.log
    timeout -k 10 600 python bench.py > gpurun_out/bench_r05g.log 2>&1
    ;;
  C)
    STEPS="smoke tests bench" bash scripts/gpu_round.sh > gpurun_out/final_c.log 2>&1
    grep -q ALLDONE gpurun_out/final_c.log
    ;;
  ALL)  # A, the c4 c5 profiles, the PMC summaries of this library (for the bench's traffic), C
    bash scripts/gpu_sort_ab.sh
    CFGS="c2 c3 c3q20 c4 c5" bash scripts/profile_round.sh > gpurun_out/final_prof.log 2>&1
    grep -q PROFILES_DONE gpurun_out/final_prof.log
    bash scripts/pmc_json_r05.sh
    STEPS="smoke tests bench" bash scripts/gpu_round.sh > gpurun_out/final_c.log 2>&1
    grep -q ALLDONE gpurun_out/final_c.log
    ;;
esac
