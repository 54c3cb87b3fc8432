set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 10 > gpurun_out/bench_pages4k.json 2> gpurun_out/bench_pages4k.err && \
timeout -k 10 300 python bench.py --workload pages8k --steps 30 --cpu-seconds 3 > gpurun_out/bench_pages8k.json 2>> gpurun_out/bench.err && \
timeout -k 10 300 python bench.py --workload zipf --steps 20 --cpu-seconds 3 > gpurun_out/bench_zipf.json 2>> gpurun_out/bench.err && \
timeout -k 10 300 python bench.py --workload chunks --steps 20 --cpu-seconds 3 > gpurun_out/bench_chunks.json 2>> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pages4k -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/prof_pages4k.log 2>&1
echo exit=$?
tail -3 gpurun_out/pytest_gpu.txt; cat gpurun_out/smoke.txt; cat gpurun_out/bench_*.json
