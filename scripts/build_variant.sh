#!/bin/bash
# Build libbasecount_hip.so with extra compiler flags into OUT (A/B variants for scripts/ab_libs.sh):
#   SRC=basecount_amd/csrc OUT=scripts/tmp/libX.so bash scripts/build_variant.sh -DFOO=1
set -e
SRC="${SRC:-basecount_amd/csrc}"; OUT="${OUT:?}"
ROCM=/opt/rocm
$ROCM/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -Wall -Wno-unused-parameter -I"$SRC/../../include" "$@" -shared -o "$OUT" \
  "$SRC"/bc_kernels.hip "$SRC"/bc_pileup.hip "$SRC"/bc_sum.hip "$SRC"/bc_rc.hip "$SRC"/bc_index.hip "$SRC"/bc_sort.hip "$SRC"/bc_capi.hip "$SRC"/bc_comm.hip \
  -L$ROCM/lib -lrccl -Wl,-rpath,$ROCM/lib 2>&1 | grep -v hip-link || true
