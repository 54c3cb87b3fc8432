#!/bin/bash
# development: k_xlong with 768-thread workgroups (9 producers + 3 chains): three steps in flight (x3a) or two (x3b), against head (xl2)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_x3a.so timeout -k 10 300 python -u -m pytest tests/test_xxh3.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4o.log 2>&1 || { tail -20 gpurun_out/t4o.log; exit 1; }
tail -1 gpurun_out/t4o.log
LWAVES=12 LCHAINS=3 FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_x3t.so timeout -k 10 120 python tools/probe_ltimes.py
for L in xl2 x3a x3b xl2 x3a x3b; do echo $L; FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 120 python tools/probe_xxh3.py chunks "16384 x"; done
WL="xxh3-chunks" LIBS="xl2 x3a" NPASS=2 bash tools/gpu_benchprofab.sh
