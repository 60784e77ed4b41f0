#!/bin/bash
# k_rc time against the batch's read count at C3's shape (BC_BENCH_READS, diagnostic): how much
# of a step is the last, partly filled round of chunks (768 resident blocks of 256 reads).
#   READS="786432 983040 1000000 1179648" bash scripts/reads_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in ${READS:-786432 983040 1000000 1179648}; do
  out=$(BC_BENCH_READS=$n timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-extras --no-e2e --steps 200 --warmup 20 ${BENCH_ARGS}) || { echo "FAILED $n"; exit 1; }
  echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step']*1e3,2), 'us/step', {k[:40]: round(x,2) for k,x in d['kernel_us'].items()}, 'parity', d['parity_vs_oracle'])"
done
