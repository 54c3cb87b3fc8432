# A/B of the varlen engine: previous build (libfdb_crc32c_prev.so) vs current, interleaved (development)
for i in 1 2; do
  for L in libfdb_crc32c_prev libfdb_crc32c; do
    echo "== $L"
    FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py ${PROBES:-4096 16384 zipf chunks} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
