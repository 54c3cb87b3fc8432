#!/bin/bash
# development: packets walk header window: two aligned chunks (w64c2) or one at the header (w64c1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c.so timeout -k 10 300 python -u -m pytest tests/test_packets.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4q.log 2>&1 || { tail -20 gpurun_out/t4q.log; exit 1; }
tail -1 gpurun_out/t4q.log
WL="packets-verify" LIBS="w64c2 w64c1" NPASS=2 bash tools/gpu_benchprofab.sh
