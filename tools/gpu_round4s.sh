#!/bin/bash
# development: XCD-parity weights in k_xxh3_rows (px: 33/31) against equal (p0: 32/32)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c.so timeout -k 10 300 python -u -m pytest tests/test_xxh3.py tests/test_pagecheck.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4s.log 2>&1 || { tail -20 gpurun_out/t4s.log; exit 1; }
tail -1 gpurun_out/t4s.log
WL="diskqueue-verify xxh3-pages4k" LIBS="" NPASS=0 true
