#!/bin/bash
# development (round 4): sparse split mode + tail cost / weight A/B
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_x16.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_xxh3.py tests/test_packets.py > gpurun_out/t16.log 2>&1 || { tail -5 gpurun_out/t16.log; exit 1; }
tail -1 gpurun_out/t16.log
ARGS="zipf chunks" LIBS="x12 x14 x14b x14c x14d x15 x16" NPASS=2 bash tools/gpu_xprobe.sh 2>&1 | grep -E "==|xxh3 (zipf  |chunks)|vrows" || exit 1
FDBCRC_LIB=$L/libfdb_crc32c_x16t.so timeout -k 10 200 python3 tools/probe_vtimes.py zipf 2>&1 | grep -E " rows| tail| end|wg" || exit 1
