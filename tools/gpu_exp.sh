#!/bin/bash
# development: interleaved A/B of engine builds (LIBS) on probe_varlen cases (PROBES), REPS passes
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pl
for rep in $(seq ${NPASS:-2}); do
for L in ${LIBS:-base}; do
  d=gpurun_out/pl/${L}_$rep
  FDBCRC_LIB=$PWD/foundationdb_amd/lib/libfdb_crc32c_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python tools/probe_varlen.py ${PROBES:-zipf} > $d.log 2>&1 || exit 1
  echo "== $L $rep: $(grep -v amdgpu.ids $d.log | tail -1)"
  python - $d/k_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "splitmix" not in r["Name"] and "rocclr" not in r["Name"]]
print("   ", "; ".join(f'{r["Name"].split("(")[0].split("::")[-1][:14]} {float(r["AverageNs"])/1000:.1f}' for r in rows[:6]))
PY
done; done
