#!/bin/bash
# development (round 4): DiskQueue lookup3 on a side stream (dq1) vs HEAD (h16)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_dq4.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_pagecheck.py tests/test_gpu_parity.py -k "diskqueue or pagecheck or verify" > gpurun_out/tdq.log 2>&1 || { tail -5 gpurun_out/tdq.log; exit 1; }
tail -1 gpurun_out/tdq.log
WL="diskqueue-verify" LIBS="h16 dq4" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
