# timing of experiment builds (wrong results by design; development only)
for L in libfdb_crc32c libfdb_crc32c_exp2 libfdb_crc32c_exp8 libfdb_crc32c_exp16; do
  echo "== $L"
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py 4096 64 1024 zipf chunks 2>&1 | grep -v amdgpu.ids || exit 1
done
