#!/bin/bash
# round-3 step B: the extent route's GPU tests, then the zipf / chunks bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -x --timeout 200 --timeout-method thread -k "extent" > gpurun_out/pytest_extent.txt 2>&1
rc=$?
tail -5 gpurun_out/pytest_extent.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload zipf --cpu-seconds 0 > gpurun_out/bench_zipf.json 2>gpurun_out/bench_zipf.err || exit 7
cat gpurun_out/bench_zipf.json
timeout -k 10 300 python -u bench.py --workload chunks --cpu-seconds 0 > gpurun_out/bench_chunks.json 2>gpurun_out/bench_chunks.err || exit 8
cat gpurun_out/bench_chunks.json
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.txt
exit $rc
