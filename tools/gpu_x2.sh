#!/bin/bash
# development: chunks on the extent route vs the block route, zipf, rocprof kernel times
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x2
for rep in 1 2; do
for R in ext blk; do
  d=gpurun_out/x2/${R}_$rep
  RT=3; [ $R = blk ] && RT=2
  FDBCRC_ROUTE=$RT timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python tools/probe_varlen.py ${PROBES:-chunks} > $d.log 2>&1 || exit 1
  echo "== $R $rep: $(grep -E 'GB/s' $d.log | tr '\n' '|')"
  python - $d/k_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"]]
print("   ", "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:14]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:7]))
PY
done; done
