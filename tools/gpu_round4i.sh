#!/bin/bash
# development (round 4): fused planner up to 2048 tiles (fu2k) vs HEAD (h9), bench protocol
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_fu2k.so timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_xxh3.py tests/test_packets.py > gpurun_out/tfu.log 2>&1 || { tail -5 gpurun_out/tfu.log; exit 1; }
tail -1 gpurun_out/tfu.log
WL="xxh3-zipf packets-verify" LIBS="h9 fu2k" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
