# A/B of several engine builds (development): LIBS="base s256" PROBES="zipf" bash tools/ab_multi.sh
for i in 1 2; do
  for L in ${LIBS:-base}; do
    echo "== $L"
    FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 120 python tools/probe_varlen.py ${PROBES:-zipf} 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
