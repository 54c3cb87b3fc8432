# development: one GPU step
export TMPDIR=/tmp
mkdir -p gpurun_out/r2f
timeout -k 10 120 python tools/dump_varlen.py || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2f/pytest_gpu.txt 2>&1; rc=$?
tail -40 gpurun_out/r2f/pytest_gpu.txt | grep -E "PASS|FAIL|Error|passed|failed" | tail -12
[ $rc -eq 0 ] || exit $rc
for L in libfdb_crc32c_v7 libfdb_crc32c; do echo "== $L"; FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py 2>&1 | grep -v amdgpu.ids || exit 1; done
