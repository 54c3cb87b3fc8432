#!/bin/bash
# development: packets walk with register-staged frame lists (pk) against HEAD's library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_pk.so timeout -k 10 300 python -u -m pytest tests/test_packets.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4p.log 2>&1 || { tail -20 gpurun_out/t4p.log; exit 1; }
tail -1 gpurun_out/t4p.log
WL="packets-verify" LIBS="main pk" NPASS=2 bash tools/gpu_benchprofab.sh
