#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for S in 1 8; do for AB in 0 3 11 27 24 4 28; do
  echo "c2 S=$S ablate=$AB $(BC_TILE_WAVES=$S BC_ABLATE=$AB timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --steps 100 --warmup 3 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["pileup_kernel_us"],1), round(d["ms_per_step"]*1e3,1))')" || exit 1
done; done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
BC_TILE_WAVES=8 BC_ABLATE=27 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof27 -o run -- python bench.py --no-cpu-baseline --steps 100 --warmup 3 > /dev/null 2>&1
cat gpurun_out/prof27/run_kernel_stats.csv | cut -c1-160
