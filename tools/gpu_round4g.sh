#!/bin/bash
# development (round 4): extent grabs of 16 blocks (gm16) vs 8 (h16)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_gm16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -k "extent or exact or route or varlen" > gpurun_out/tgm.log 2>&1 || { tail -5 gpurun_out/tgm.log; exit 1; }
tail -1 gpurun_out/tgm.log
WL="zipf" LIBS="h16 gm16" NPASS=3 bash tools/gpu_benchprofab.sh || exit 1
