#!/bin/bash
# development: k_xlong variants (xl2: vmcnt fix; xl4: + next buffer opened once the current is claimed)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_xl4.so timeout -k 10 300 python -u -m pytest tests/test_xxh3.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t4n.log 2>&1 || { tail -20 gpurun_out/t4n.log; exit 1; }
tail -1 gpurun_out/t4n.log
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_lt4.so timeout -k 10 120 python tools/probe_ltimes.py
for L in xl2 xl4 xl2 xl4; do echo $L; FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 120 python tools/probe_xxh3.py chunks "16384 x" "rand 4-16K"; done
WL="xxh3-chunks" LIBS="pw xl4" NPASS=2 bash tools/gpu_benchprofab.sh
