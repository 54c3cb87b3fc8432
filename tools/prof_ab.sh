# development: interleaved rocprofv3 kernel averages of pmc_probe modes ($MODES) for engine builds ($LIBS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
n=0
for rep in 1 2; do
for M in ${MODES:-pages4k}; do
for L in ${LIBS:-base}; do
  n=$((n+1)); d=gpurun_out/ab/${M}_${L}_$rep
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python tools/pmc_probe.py $M > $d.log 2>&1 || exit 1
  python - $d/k_kernel_stats.csv "$M $L $rep" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"]]
print(sys.argv[2], "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:18]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:4]))
PY
done; done; done
