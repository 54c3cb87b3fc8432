# Development: XXH3 varlen probes with kernel stats, per library ($LIBS, default the
# current one).  ARGS = probe filters.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/xp
for rep in $(seq ${NPASS:-1}); do
for L in ${LIBS:-cur}; do
  lib=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so
  [ "$L" = cur ] && lib=$PWD/foundationdb_amd/lib/libfdb_crc32c.so
  d=gpurun_out/xp/${L}_$rep
  FDBCRC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/probe_xxh3.py $ARGS > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "== $L"
  grep "^xxh3" $d.log
  python3 - $d/run_kernel_stats.csv <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if "splitmix" in r['Name']: continue
    print(f"   {r['Name'][:50]:50s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
done
