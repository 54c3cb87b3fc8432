set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for L in r2 r4; do
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 200 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$L.txt 2>&1 || { tail -20 gpurun_out/pytest_$L.txt; exit 1; }
  tail -1 gpurun_out/pytest_$L.txt
done
for i in 1 2; do
  for L in base r2 r4; do
    echo "== $L"
    FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 120 python tools/probe_varlen.py 4096 64 zipf chunks 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
