#!/bin/bash
# round 3: extent route parity, then zipf / chunks bench lines and kernel stats
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -x --timeout 200 --timeout-method thread -k "extent or varlen_configs or route_choice" > gpurun_out/pytest_extent.txt 2>&1
rc=$?
tail -8 gpurun_out/pytest_extent.txt
[ $rc -ne 0 ] && exit $rc
for w in zipf chunks; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds 0 > gpurun_out/bench_$w.json 2>gpurun_out/bench_$w.err || exit 7
  cat gpurun_out/bench_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:30], d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_ok'])"
done
CFGS="3:4096" WORKLOADS="zipf chunks" bash tools/prof_routes.sh || exit 1
