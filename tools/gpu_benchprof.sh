#!/bin/bash
# development: rocprofv3 kernel stats of bench.py runs ($WL)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bp
for w in ${WL:-zipf}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bp/$w -o k -- python bench.py --workload $w --steps 20 --cpu-seconds 0 > gpurun_out/bp/$w.json 2> gpurun_out/bp/$w.err || { tail -3 gpurun_out/bp/$w.err; exit 1; }
  python - gpurun_out/bp/$w/k_kernel_stats.csv $w <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"]]
print(sys.argv[2], "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:16]} n={r["Calls"]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:8]))
PY
done
