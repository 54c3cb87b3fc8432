#!/bin/bash
# development (round 4): 1024-buffer planner tiles (x17) vs HEAD (h16)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_x17.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_xxh3.py tests/test_packets.py > gpurun_out/t17.log 2>&1 || { tail -5 gpurun_out/t17.log; exit 1; }
tail -1 gpurun_out/t17.log
ARGS="zipf chunks 64 " LIBS="h16 x17" NPASS=2 bash tools/gpu_xprobe.sh 2>&1 | grep -E "==|xxh3 (zipf  |chunks|64 )|k_x" || exit 1
WL="xxh3-zipf xxh3-chunks" LIBS="h16 x17" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
