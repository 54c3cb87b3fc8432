#!/bin/bash
# round 3 iteration: parity subset (TESTS -k expression), bench lines (BENCH), kernel stats (PROF, PROFX3)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_xxh3.py tests/test_gpu_parity.py tests/test_pagecheck.py -v -x --timeout 200 --timeout-method thread -m gpu -k "${TESTS:-xxh3 or extent or varlen_configs or route_choice}" > gpurun_out/pytest_iter.txt 2>&1
rc=$?
tail -4 gpurun_out/pytest_iter.txt
[ $rc -ne 0 ] && exit $rc
for w in ${BENCH:-zipf chunks xxh3-chunks xxh3-zipf}; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds 0 > gpurun_out/bench_$w.json 2>gpurun_out/bench_$w.err || exit 7
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$w.json').read()); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_ok'])"
done
[ -n "$PROF" ] && { CFGS="${CFGS:-3:4096}" WORKLOADS="$PROF" bash tools/prof_routes.sh || exit 1; }
[ -n "$PROFX3" ] && { WORKLOADS="$PROFX3" bash tools/prof_quick.sh || exit 1; }
[ -n "$PMCMODES" ] && { MODES="$PMCMODES" bash tools/pmc_quick.sh || exit 1; }
exit 0
