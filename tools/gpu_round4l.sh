#!/bin/bash
# development (round 4): XCD-parity weighted page ranges (pw, pw2) vs HEAD (h12)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_pw.so timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests > gpurun_out/tpw.log 2>&1 || { tail -5 gpurun_out/tpw.log; exit 1; }
tail -1 gpurun_out/tpw.log
FDBCRC_LIB=$L/libfdb_crc32c_pwt.so timeout -k 10 200 python3 tools/probe_ptimes.py || exit 1
WL="pages4k pages8k" LIBS="h12 pw pw2" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
