#!/bin/bash
# development (round 4): generation-weighted ranges in k_xxh3_rows (xr) vs HEAD (h11)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_xr2.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_pagecheck.py > gpurun_out/txr.log 2>&1 || { tail -5 gpurun_out/txr.log; exit 1; }
tail -1 gpurun_out/txr.log
FDBCRC_LIB=$L/libfdb_crc32c_xr2t.so timeout -k 10 200 python3 tools/probe_rtimes.py || exit 1
WL="xxh3-pages4k diskqueue-verify sqlite-verify" LIBS="xr xr2 xr3" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
