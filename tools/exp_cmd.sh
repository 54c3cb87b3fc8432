set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for L in ${LIBS:-libfdb_crc32c libfdb_crc32c_v4}; do
  echo "== $L"
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py ${PROBES:-} 2>&1 | grep -v amdgpu.ids || exit 1
done
for W in zipf; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$W -o $W -- python tools/probe_varlen.py "$W" > gpurun_out/ks_$W.log 2>&1 || exit 1
echo "== $W"; cut -d, -f1-4 gpurun_out/ks_$W/${W}_kernel_stats.csv | cut -c1-110 | grep -v "splitmix\|Name"
done
