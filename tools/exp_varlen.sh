for L in libfdb_crc32c libfdb_crc32c_exp1 libfdb_crc32c_exp2 libfdb_crc32c_exp4 libfdb_crc32c_exp7; do
  echo "== $L"
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py 4096 16384 chunks zipf 2>&1 | grep -v amdgpu.ids || exit 1
done
