# development: texture-address / L1 pressure of the page kernel and the window engine
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/pmcta
mkdir -p $P
for MODE in ${MODES:-pages4k zipf chunks}; do
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $P/$MODE -o a_$MODE -- python tools/pmc_probe.py $MODE > $P/$MODE.log 2>&1 || exit 1
  python - $P/$MODE/a_${MODE}_counter_collection.csv <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
done
