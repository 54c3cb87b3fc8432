set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_t768.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu768.txt 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu768.txt
[ $rc -eq 0 ] || exit $rc
for L in ${LIBS:-libfdb_crc32c libfdb_crc32c_t768}; do
  echo "== $L"
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py ${PROBES:-} 2>&1 | grep -v amdgpu.ids || exit 1
done
