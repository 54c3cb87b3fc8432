export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_redwood.py > gpurun_out/t/rw.log 2>&1; rc=$?; tail -30 gpurun_out/t/rw.log; [ $rc -eq 0 ] || exit $rc
for w in redwood-verify redwood-seal; do
timeout -k 10 300 python bench.py --workload $w --steps 20 --cpu-seconds 3 > gpurun_out/t/$w.json 2> gpurun_out/t/$w.err || { tail -20 gpurun_out/t/$w.err; exit 1; }
cut -c1-400 gpurun_out/t/$w.json
done
