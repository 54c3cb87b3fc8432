#!/bin/bash
# development: rocprofv3 kernel stats of bench.py runs ($WL) for engine builds ($LIBS), same box
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bpab
for rep in $(seq ${NPASS:-1}); do
for w in ${WL:-zipf}; do
for L in ${LIBS:-new}; do
  d=gpurun_out/bpab/${w}_${L}_$rep
  LL=${L%%+*}; XS=0; [ "$L" != "$LL" ] && XS=1   # "name+static": FDBCRC_XSTATIC=1
  FDBCRC_XSTATIC=$XS FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$LL.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python bench.py --workload $w --steps 20 --cpu-seconds 0 ${BENCH_EXTRA:-} > $d.json 2> $d.err || { tail -3 $d.err; exit 1; }
  python - $d/k_kernel_stats.csv "$w $L" $d.json <<'PY'
import csv, sys, json
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"] and int(r["Calls"]) > 2]
d = json.load(open(sys.argv[3]))
print(sys.argv[2], d["ms_per_step"], "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:16]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:8]))
PY
done; done; done
