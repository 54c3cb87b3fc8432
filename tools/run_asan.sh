#!/bin/bash
# Non-GPU test suite against the ASan + UBSan build of the host code
# (make asan): scalar crc32c_append (SSE4.2 and forced-software paths),
# GF(2) helpers, the write checker's bookkeeping, argument validation.
# The Python interpreter is not instrumented, so libasan is preloaded and leak
# checking is off (CPython's allocator is not ours); UBSan aborts on the first
# finding (-fno-sanitize-recover).
set -e
cd "$(dirname "$0")/.."
make -s asan
export LD_PRELOAD=$(g++ -print-file-name=libasan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_asan.so
python -m pytest -x -q -m "not gpu" tests/test_boundary.py tests/test_write_checker.py tests/test_host_scalar.py "$@"
