# development: one GPU step
export TMPDIR=/tmp
for L in libfdb_crc32c libfdb_crc32c_v8; do echo "== $L"; FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py "1 MiB" 16384 4096 zipf chunks 2>&1 | grep -v amdgpu.ids || exit 1; done
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_v8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
