#!/bin/bash
# A/B of the summary fold: the in-tree library vs scripts/tmp/lib_oldfold.so (round-4 fold).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIB=basecount_amd/libbasecount_hip.so
cp $LIB /tmp/lib_cur.so
for v in cur old cur old; do
  if [ $v = old ]; then cp scripts/tmp/lib_oldfold.so $LIB; else cp /tmp/lib_cur.so $LIB; fi
  echo "== $v"
  timeout -k 10 120 python scripts/micro/fold_bench.py || { cp /tmp/lib_cur.so $LIB; exit 1; }
done
cp /tmp/lib_cur.so $LIB
