export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for L in "" ${LIBS:-}; do
  lib=""; [ -n "$L" ] && lib=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so
  d=gpurun_out/ab/nv-${L:-prod}
  FDBCRC_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python bench.py --workload xxh3-chained --steps 20 --cpu-seconds 0 --no-verify > $d.json 2> $d.err || { tail -3 $d.err; exit 1; }
  python - $d/k_kernel_stats.csv "${L:-prod}" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if int(r["Calls"]) > 2]
print(sys.argv[2], "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:14]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:4]))
PY
done
