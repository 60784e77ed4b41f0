#!/bin/bash
# Summary-fold variants A/B on crafted partials (scripts/micro/fold_bench.py): the in-tree library
# against scripts/tmp/lib_*.so (VARIANTS), alternating, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cp basecount_amd/libbasecount_hip.so /tmp/lib_cur.so
for rep in 1 2; do
  for v in cur ${VARIANTS:-binade oldload}; do
    if [ $v = cur ]; then cp /tmp/lib_cur.so basecount_amd/libbasecount_hip.so; else cp scripts/tmp/lib_$v.so basecount_amd/libbasecount_hip.so; fi
    echo "== $v"; timeout -k 10 200 python scripts/micro/fold_bench.py || { cp /tmp/lib_cur.so basecount_amd/libbasecount_hip.so; exit 1; }
  done
done
cp /tmp/lib_cur.so basecount_amd/libbasecount_hip.so
