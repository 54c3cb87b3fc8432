#!/bin/bash
# development (round 4): planner/tail knobs under the bench protocol
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_qm512.so timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_xxh3.py > gpurun_out/tqm.log 2>&1 || { tail -5 gpurun_out/tqm.log; exit 1; }
tail -1 gpurun_out/tqm.log
WL="xxh3-zipf" LIBS="h9 tc768 tc1024 qm512 ow23" NPASS=3 bash tools/gpu_benchprofab.sh || exit 1
