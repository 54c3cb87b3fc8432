#!/bin/bash
# development: k_xcount's neighbour metadata loaded directly (xc) against HEAD's library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_xc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "extent or varlen or zipf" > gpurun_out/t4r.log 2>&1 || { tail -20 gpurun_out/t4r.log; exit 1; }
tail -1 gpurun_out/t4r.log
WL="zipf" LIBS="main xc" NPASS=2 bash tools/gpu_benchprofab.sh
