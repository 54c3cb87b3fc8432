# development: rocprofv3 kernel averages of probe_varlen cases ($PROBES) for several engine builds ($LIBS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pl
for L in ${LIBS:-base}; do
  d=gpurun_out/pl/$L
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python tools/probe_varlen.py ${PROBES:-zipf} > $d.log 2>&1 || exit 1
  echo "== $L"; grep -v amdgpu.ids $d.log | tail -3
  cut -d, -f1-4 $d/k_kernel_stats.csv | grep -v splitmix | head -6
done
