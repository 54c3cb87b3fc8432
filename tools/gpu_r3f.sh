#!/bin/bash
# round 3 (second half): tests named by TESTK, bench lines of WORKLOADS, kernel stats
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTF:-tests/test_xxh3.py} -v -x --timeout 200 --timeout-method thread -k "${TESTK:-xxh3}" > gpurun_out/pytest_r3f.txt 2>&1
rc=$?
tail -6 gpurun_out/pytest_r3f.txt
[ $rc -ne 0 ] && exit $rc
for w in ${WORKLOADS:-xxh3-chunks}; do
  timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds 0 > gpurun_out/bench_$w.json 2>gpurun_out/bench_$w.err || exit 7
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$w.json').read()); print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_ok'])"
done
[ -n "$NOPROF" ] && exit 0
WORKLOADS="${PWORKLOADS:-$WORKLOADS}" bash tools/prof_quick.sh || exit 1
