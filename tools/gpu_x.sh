#!/bin/bash
# development: extent-route GPU tests, then rocprof kernel times of probe cases
# ($PROBES) with the dynamic grab kernel and with static ranges (FDBCRC_XSTATIC=1)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/x
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS ${KEXPR:+-k "$KEXPR"} > gpurun_out/x/tests.log 2>&1
  rc=$?; tail -4 gpurun_out/x/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
for M in ${MODES:-grab static}; do
  d=gpurun_out/x/${M}_$rep
  XS=0; [ $M = static ] && XS=1
  FDBCRC_XSTATIC=$XS timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python tools/probe_varlen.py ${PROBES:-zipf} > $d.log 2>&1 || exit 1
  echo "== $M $rep: $(grep -E 'GB/s' $d.log | tr '\n' '|')"
  python - $d/k_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"]]
print("   ", "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:14]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:7]))
PY
done; done
