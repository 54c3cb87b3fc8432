#!/bin/bash
# development: the extent route's GPU tests, then zipf bench + rocprofv3 kernel stats (fused and, with AB=1, FDBX_FUSED=0)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_xxh3.py -k "${KEXPR:-extent or varlen or route or zipf or chunks}" > gpurun_out/x/tests.log 2>&1; rc=$?; tail -5 gpurun_out/x/tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARS:-1 0 1 0}; do
  FDBX_FUSED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x/p$v -o k -- python bench.py --workload zipf --steps 20 --cpu-seconds 0 > gpurun_out/x/zipf$v.json 2> gpurun_out/x/zipf$v.err || { tail -5 gpurun_out/x/zipf$v.err; exit 1; }
  python - gpurun_out/x/p$v/k_kernel_stats.csv $v gpurun_out/x/zipf$v.json <<'PY'
import csv, sys, json
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"]]
d = json.load(open(sys.argv[3]))
print("fused=" + sys.argv[2], d["ms_per_step"], d["roofline"]["frac"], d["parity_ok"], "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:12]} n={r["Calls"]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:6]))
PY
done
