# development: one SQ PMC pass per mode ($MODES) -> per-kernel counter means
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmq
for m in ${MODES:-chunks}; do
  timeout -s KILL 120 rocprofv3 --pmc ${PMC:-GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES} --kernel-trace --output-format csv -d gpurun_out/pmq/$m -o sq -- python tools/pmc_probe.py $m > gpurun_out/pmq/$m.log 2>&1 || exit 1
  python - "$m" <<'PY'
import csv, collections, glob, sys
m = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/pmq/{m}/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"][:34], r["Counter_Name"])].append(float(r["Counter_Value"]))
ks = sorted({k for k, _ in agg})
for k in ks:
    print(m, k, {c: round(sum(v) / len(v)) for (kk, c), v in agg.items() if kk == k})
PY
done
