#!/bin/bash
# C5 kernel durations (rocprofv3 kernel trace, one stream) for the in-tree library and an older one
# (OLD=path): the fold / summary kernels compared.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=basecount_amd/libbasecount_hip.so
cp $LIB /tmp/lib_cur.so
for v in cur old; do
  if [ $v = old ]; then cp "${OLD:?}" $LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5_$v -o run -- \
    python bench.py --config c5 --no-cpu-baseline --no-extras --no-e2e --lean --launch eager --steps 5 --warmup 1 \
    --streams 1 > gpurun_out/prof5_$v.log 2>&1
  rc=$?; echo "prof $v rc=$rc"; [ $rc -eq 0 ] || { cp /tmp/lib_cur.so $LIB; exit $rc; }
done
cp /tmp/lib_cur.so $LIB
echo ALLDONE
