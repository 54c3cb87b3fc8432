# development: rocprofv3 kernel averages of the page probe (1 Mi x 4 KiB) for several engine builds ($LIBS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
for L in ${LIBS:-base}; do
  d=gpurun_out/pp/$L
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python tools/pmc_probe.py ${MODE:-pages4k} > $d.log 2>&1 || exit 1
  echo "== $L"
  cut -d, -f1-4 $d/k_kernel_stats.csv | grep -v splitmix | head -4
done
