#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "fused or kernel1 or full_size or smoke" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log
case $rc in 124|134|137|139) exit $rc;; esac
for C in c2 c3; do for S in 4 8; do for AB in 0 3; do
  st=100; [ $C = c3 ] && st=20
  echo "$C S=$S ab=$AB $(BC_ABLATE=$AB BC_TILE_WAVES=$S timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --steps $st --warmup 3 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["pileup_kernel_us"],1), round(d["ms_per_step"]*1e3,1), d["parity_vs_oracle"])')" || exit 1
done; done; done
