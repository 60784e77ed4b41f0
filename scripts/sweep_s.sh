#!/bin/bash
# Waves-per-tile sweep (bench.py --tile-waves): CFGS="c2 c3" SS="2 4 8" bash scripts/sweep_s.sh
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for C in ${CFGS:-c2 c3}; do for S in ${SS:-2 4 8}; do
  timeout -k 10 300 python bench.py --tile-waves $S --config $C --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/sw_${C}_$S.log 2>&1
  rc=$?; case $rc in 124|134|137|139) echo "FATAL $rc"; exit $rc;; esac
  python3 -c "import json; l=[x for x in open('gpurun_out/sw_${C}_$S.log') if x.startswith('{')]; d=json.loads(l[-1]) if l else {}; print('$C S=$S', round(d.get('device_us_per_step',-1),2), d.get('kernel_us'), 'parity', d.get('parity_vs_oracle'))"
done; done
