#!/bin/bash
# development (round 4): k_bigblocks work stealing (bs) vs HEAD (h16)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/foundationdb_amd/lib
for lib in bs h16 bs h16; do
  FDBCRC_LIB=$L/libfdb_crc32c_$lib.so timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread tests/test_gpu_parity.py -k "route or block or chunks or varlen" > gpurun_out/tbs_$lib.log 2>&1; echo "$lib rc=$? $(tail -1 gpurun_out/tbs_$lib.log)"
done
FDBCRC_LIB=$L/libfdb_crc32c_bst.so timeout -k 10 200 python3 tools/probe_btimes.py chunks || exit 1
WL="chunks" LIBS="h16 bs" NPASS=2 bash tools/gpu_benchprofab.sh || exit 1
