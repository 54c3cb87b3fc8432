# Full evidence run (GPU box): parity tests, bench lines (all workloads, CPU
# baselines), rocprofv3 kernel-trace summary of the headline bench command and
# PMC passes.  Outputs under gpurun_out/round/, copied into profiles/<round>/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=gpurun_out/round
mkdir -p $R
timeout -k 10 300 python -m pytest tests -m gpu -q > $R/pytest_gpu.txt 2>&1 || { tail -5 $R/pytest_gpu.txt; exit 1; }
tail -1 $R/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $R/bench_pages4k.json 2> $R/bench_pages4k.err || exit 1
for w in pages8k zipf chunks chunks-host; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --cpu-seconds 5 > $R/bench_$w.json 2> $R/bench_$w.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_pages4k -o pages4k -- python bench.py --cpu-seconds 0 > $R/prof_pages4k.log 2>&1 || exit 1
for w in zipf chunks; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$w -o $w -- python bench.py --workload $w --steps 20 --cpu-seconds 0 > $R/prof_$w.log 2>&1 || exit 1
done
P=gpurun_out/pmc
mkdir -p $P
for MODE in pages4k stride0; do
  for spec in "fetch FETCH_SIZE" "write WRITE_SIZE" "sq GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES" "sq2 GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
    set -- $spec; name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $P/$MODE -o ${name}_$MODE -- python tools/pmc_probe.py $MODE > $P/$MODE.log 2>&1 || exit 1
  done
done
cat $R/bench_*.json | cut -c1-400
