#!/bin/bash
# development: packets walk frames staged per flush: 8 (main), 16, 32
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_s32.so timeout -k 10 300 python -u -m pytest tests/test_packets.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4q.log 2>&1 || { tail -20 gpurun_out/t4q.log; exit 1; }
tail -1 gpurun_out/t4q.log
WL="packets-verify" LIBS="main s16 s32" NPASS=2 bash tools/gpu_benchprofab.sh
