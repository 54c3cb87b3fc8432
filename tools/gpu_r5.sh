#!/bin/bash
# round-5 development runs on one GPU box:
#   MB=1     the load-shape microbenchmark (tools/membench3)
#   TLIB=x   the GPU tests in $T against libfdb_crc32c_x.so
#   WL, LIBS same-box A/B of bench lines (tools/gpu_benchprofab.sh)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$MB" ]; then
  timeout -k 10 120 ./tools/membench3 > gpurun_out/mb3.log 2>&1 && cat gpurun_out/mb3.log || exit 1
fi
if [ -n "$TLIB" ]; then
  for L in $TLIB; do
    FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 500 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/t5_$L.log 2>&1; rc=$?
    echo "== tests $L rc=$rc"; tail -4 gpurun_out/t5_$L.log
    [ $rc -eq 0 ] || exit $rc
  done
fi
if [ -n "$WL" ]; then
  bash tools/gpu_benchprofab.sh || exit 1
fi
