for L in libfdb_crc32c libfdb_crc32c_exp8 libfdb_crc32c_exp16 libfdb_crc32c_exp2; do
  echo "== $L"
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/$L.so timeout -k 10 120 python tools/probe_varlen.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 200 python bench.py --workload pages4k-host --steps 5 --warmup 2 --cpu-seconds 2 > gpurun_out/bench_pages4k-host.json 2> gpurun_out/bench_pages4k-host.err; cat gpurun_out/bench_pages4k-host.json | cut -c1-600; tail -3 gpurun_out/bench_pages4k-host.err
