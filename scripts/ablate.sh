#!/bin/bash
# Kernel-time ablations (BC_ABLATE bits, diagnostic only): ABL="0 4 32" CFGS="c2 c3" bash scripts/ablate.sh
# Needs the diagnostic build: make -C basecount_amd/csrc -B DIAG=1 (rebuild without DIAG afterwards).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for c in ${CFGS:-c2 c3}; do for a in ${ABL:-0 4 32 1}; do
  BC_ABLATE=$a timeout -k 10 300 python bench.py --allow-diag --config $c --no-cpu-baseline --steps 50 --warmup 5 ${BENCH_ARGS} > gpurun_out/abl_${c}_$a.log 2>&1
  rc=$?; case $rc in 124|134|137|139) echo "FATAL $rc"; exit $rc;; esac
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/abl_${c}_$a.log') if x.startswith('{')]; d=json.loads(l[-1]) if l else {}; print('$c ablate $a', round(d.get('device_us_per_step',-1),2), d.get('kernel_us'), 'parity', d.get('parity_vs_oracle'))"
done; done
