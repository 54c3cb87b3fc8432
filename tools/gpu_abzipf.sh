#!/bin/bash
# development: same-box A/B of bench lines ($WL, default zipf) over libraries
# ($LIBS: "" = the product library, NAME = libfdb_crc32c_NAME.so, NAME:ENV=V to
# add an environment setting), rocprofv3 kernel stats per pass; optional GPU
# tests ($TESTK: pytest -k expression) against the first experiment library.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
if [ -n "$TESTK" ]; then
  L=${TLIB:-}
  FDBCRC_LIB=${L:+$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so} timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests -k "$TESTK" > gpurun_out/ab/tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for pass in $(seq ${PASSES:-2}); do
for spec in ${LIBS:-prod}; do
  name=${spec%%:*}; envs=""; [ "$spec" != "$name" ] && envs=${spec#*:}
  lib=""; [ "$name" != "prod" ] && lib=$PWD/foundationdb_amd/lib/libfdb_crc32c_$name.so
  for w in ${WL:-zipf}; do
    d=gpurun_out/ab/$w-$name-$pass
    env $envs FDBCRC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python bench.py --workload $w --steps 20 --cpu-seconds 0 > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
    python - $d/k_kernel_stats.csv $d.json "$w $spec #$pass" <<'PY'
import csv, sys, json
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"] and int(r["Calls"]) > 2]
d = json.load(open(sys.argv[2]))
print(f'{sys.argv[3]:28s} ms={d["ms_per_step"]:.4f} frac={d["roofline"]["frac"]:.4f} ok={d["parity_ok"]} ' + "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:12]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:6]))
PY
  done
done
done
