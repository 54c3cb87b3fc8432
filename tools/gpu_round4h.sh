#!/bin/bash
# development (round 4): lane-per-buffer packet walk (pk1) vs HEAD (h16)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_pk2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_packets.py > gpurun_out/tpk.log 2>&1 || { tail -15 gpurun_out/tpk.log; exit 1; }
tail -1 gpurun_out/tpk.log
WL="packets-verify" LIBS="h16 pk1 pk2" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
