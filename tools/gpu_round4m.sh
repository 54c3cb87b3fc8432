#!/bin/bash
# development: XCD-parity ranges in k_xgrab/k_bigblocks (pw3) — parity tests, then bench A/B against pw (pages only)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_pw3.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4m.log 2>&1 || { tail -20 gpurun_out/t4m.log; exit 1; }
tail -2 gpurun_out/t4m.log
WL="zipf chunks pages4k" LIBS="pw pw3" NPASS=2 bash tools/gpu_benchprofab.sh
