# development: one GPU step
export TMPDIR=/tmp
mkdir -p gpurun_out/r2h
timeout -k 10 300 python -u -m pytest tests/test_pagecheck.py tests/test_write_checker.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2h/pytest_gpu.txt 2>&1; rc=$?
tail -12 gpurun_out/r2h/pytest_gpu.txt | grep -E "PASS|FAIL|Error|passed|failed"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload sqlite-verify --steps 20 --cpu-seconds 0 > gpurun_out/r2h/bench_sqlite-verify.json || exit 1
cut -c1-400 gpurun_out/r2h/bench_sqlite-verify.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2h/prof -o sq -- python bench.py --workload sqlite-verify --steps 10 --cpu-seconds 0 --no-verify > gpurun_out/r2h/prof.log 2>&1 || exit 1
