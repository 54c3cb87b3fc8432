set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for L in ${LIBS:-libfdb_crc32c}; do
  echo "== $L"
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py ${PROBES:-} 2>&1 | grep -v amdgpu.ids || exit 1
done
for W in zipf "64 x"; do
N=$(echo "$W" | tr -d ' ')
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$N -o $N -- python tools/probe_varlen.py "$W" > gpurun_out/ks_$N.log 2>&1 || exit 1
echo "== $W"; cut -d, -f1-4 gpurun_out/ks_$N/${N}_kernel_stats.csv | cut -c1-110 | grep -v splitmix
done
