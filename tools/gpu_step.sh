# development: one GPU step
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_xxh3.py 2>&1 | tee gpurun_out/step_probe.log
FDBCRC_LIB=foundationdb_amd/lib/libfdb_crc32c_xold.so timeout -k 10 200 python -u tools/probe_xxh3.py 2>&1 | tee gpurun_out/step_probe_old.log
