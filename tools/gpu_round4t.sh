#!/bin/bash
# development: XCD-parity weights in the XXH3 varlen planner's quanta (vx: 33/31) against unweighted (v0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_vx.so timeout -k 10 300 python -u -m pytest tests/test_xxh3.py tests/test_packets.py tests/test_pagecheck.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4t.log 2>&1 || { tail -20 gpurun_out/t4t.log; exit 1; }
tail -1 gpurun_out/t4t.log
WL="xxh3-zipf xxh3-chunks packets-verify" LIBS="v0 vx" NPASS=2 bash tools/gpu_benchprofab.sh
