#!/bin/bash
# round-3 GPU evidence step A: GPU suite, warm-up probe, default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python -u tools/probe_warmup.py 60 0 > gpurun_out/warmup0.json 2>gpurun_out/warmup0.err || exit 5
timeout -k 10 120 python -u tools/probe_warmup.py 60 2000 > gpurun_out/warmup2000.json 2>gpurun_out/warmup2000.err || exit 6
timeout -k 10 300 python -u bench.py > gpurun_out/bench_pages4k.json 2>gpurun_out/bench_pages4k.err || exit 7
cat gpurun_out/bench_pages4k.json
exit $rc
