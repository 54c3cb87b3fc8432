#!/bin/bash
# development (round 4): XXH3 tail form x older-wave weight, zipf probes, two passes
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
FDBCRC_LIB=$L/libfdb_crc32c_x14.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_xxh3.py -k "varlen or exact or split" > gpurun_out/t13.log 2>&1 || { tail -5 gpurun_out/t13.log; exit 1; }
tail -1 gpurun_out/t13.log
ARGS="zipf" LIBS="x12 x13 x14 x14b x14c x14d x15" NPASS=2 bash tools/gpu_xprobe.sh 2>&1 | grep -E "==|xxh3 (zipf  |zipf unal)" || exit 1
FDBCRC_LIB=$L/libfdb_crc32c_x14t.so timeout -k 10 200 python3 tools/probe_vtimes.py zipf 2>&1 | grep -E " rows| tail| end|wg" || exit 1
