#!/bin/bash
# development (round 4): XXH3 weighted planner + CRC extent work stealing, one box
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
L=$PWD/foundationdb_amd/lib
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_xxh3.py tests/test_packets.py tests/test_xxh3_plan.py > gpurun_out/r4a/t1.log 2>&1 || { tail -5 gpurun_out/r4a/t1.log; exit 1; }
tail -1 gpurun_out/r4a/t1.log
FDBCRC_LIB=$L/libfdb_crc32c_cs.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "extent or exact or varlen or route" > gpurun_out/r4a/t2.log 2>&1 || { tail -5 gpurun_out/r4a/t2.log; exit 1; }
tail -1 gpurun_out/r4a/t2.log
ARGS="zipf 16384 chunks" LIBS="x12 x12a x12b" bash tools/gpu_xprobe.sh 2>&1 | grep -E "==|xxh3 (zipf  |zipf unal|16384|chunks)" || exit 1
FDBCRC_LIB=$L/libfdb_crc32c_x12t.so timeout -k 10 200 python3 tools/probe_vtimes.py zipf 2>&1 | grep -E "rows|tail|end|wg" || exit 1
FDBCRC_LIB=$L/libfdb_crc32c_ct.so timeout -k 10 200 python3 tools/probe_xtimes.py zipf || exit 1
FDBCRC_LIB=$L/libfdb_crc32c_cst.so timeout -k 10 200 python3 tools/probe_xtimes.py zipf || exit 1
WL=zipf LIBS="x12 cs" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
