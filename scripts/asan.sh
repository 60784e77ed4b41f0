#!/bin/bash
# Host sanitizer run: the BAM decoder / formatter (libbcio) and the
# oracle's C restatements rebuilt with -fsanitize=address,undefined, then the CPU tests that drive
# them — the BAM round trips, hostile BGZF/BAM inputs (tests/test_bam_fuzz.py), the formatter and
# the oracle against the reference's golden vectors — run with those builds loaded.  CPU only.
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C basecount_amd/csrc asan
make -s -C oracle asan
ASAN_RT=$(gcc -print-file-name=libasan.so)
export BASECOUNT_HOST_LIB_DIR="$PWD/basecount_amd/asan"
export ORACLE_LIB_DIR="$PWD/oracle/_asan"
# CPython itself is not instrumented and keeps its arenas until exit: leaks are not reported
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
LD_PRELOAD="$ASAN_RT${LD_PRELOAD:+:$LD_PRELOAD}" \
  python -m pytest -q -p no:cacheprovider -m "not gpu" \
    tests/test_host.py tests/test_bam_fuzz.py tests/test_oracle.py "$@"
