#!/bin/bash
# round-4 final check of the in-tree library: GPU suite, smoke, headline and packets-verify lines
cd $GRAFT_REPO_ROOT
R=gpurun_out/final4
mkdir -p $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $R/pytest_gpu.txt 2>&1 || { tail -5 $R/pytest_gpu.txt; exit 1; }
tail -1 $R/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.txt 2>&1 || exit 1
tail -1 $R/smoke.txt
timeout -k 10 300 python bench.py > $R/bench_pages4k.json 2> $R/bench_pages4k.err || exit 1
timeout -k 10 300 python bench.py --workload packets-verify --steps 20 --cpu-seconds 5 > $R/bench_packets-verify.json 2> $R/bench_packets-verify.err || exit 1
for f in $R/bench_*.json; do echo "$f $(cut -c1-160 $f)"; done
