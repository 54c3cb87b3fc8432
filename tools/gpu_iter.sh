# quick iteration: GPU parity tests + headline bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for w in ${WORKLOADS:-pages4k}; do
  timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_$w.json')); print('$w', d['value'], 'GiB/s', d['pct_of_hbm_read_peak'], '% ; kernel', d['roofline']['achieved'], 'GB/s', d['roofline']['avg_launch_ms'], 'ms', 'ok' if d['parity_ok'] else 'PARITY FAIL')"
done
