# Full evidence run (GPU box): parity tests, smoke, bench lines (all
# workloads, CPU baselines), rocprofv3 kernel-trace summaries, PMC passes and
# the scalar drop-in benchmark on the box's host CPU.  Outputs under
# gpurun_out/$ROUND/ (copied into profiles/$ROUND/ afterwards).
#   gpurun -- "STAGE=1 ROUND=round2 COMMIT=$(git rev-parse --short HEAD) bash tools/profile_round.sh"  (tests, benches)
#   gpurun -- "STAGE=2 ..."  (rocprofv3 kernel traces and PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ROUND=${ROUND:-round6}
R=gpurun_out/$ROUND
P=gpurun_out/pmc
mkdir -p $R $P
echo "${COMMIT:-unknown}" > $R/commit.txt
echo "${COMMIT:-unknown}" > $P/commit.txt
if [ "${STAGE:-1}" = 1 ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $R/pytest_gpu.txt 2>&1 || { tail -5 $R/pytest_gpu.txt; exit 1; }
tail -1 $R/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > $R/bench_pages4k.json 2> $R/bench_pages4k.err || exit 1
for w in pages8k zipf zipf-scattered chunks chunks-host pages4k-host xxh3-pages4k xxh3-zipf xxh3-chunks xxh3-chained sqlite-verify sqlite-verify-host diskqueue-verify sqlite-seal diskqueue-seal packets-verify redwood-verify redwood-seal; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --cpu-seconds 5 > $R/bench_$w.json 2> $R/bench_$w.err || { tail -3 $R/bench_$w.err; exit 1; }
done
echo benches done
# the headline's first launches in a fresh process (bench.py runs --warmup 5)
timeout -k 10 120 python -u tools/probe_warmup.py 60 0 > $R/warmup0.json 2> $R/warmup0.err || exit 1
timeout -k 10 120 python -u tools/probe_warmup.py 60 2000 > $R/warmup2000.json 2> $R/warmup2000.err || exit 1
gcc -O2 -o /tmp/bench_scalar tools/bench_scalar.c -ldl && timeout -k 10 200 /tmp/bench_scalar > $R/bench_scalar.jsonl || exit 1
grep "model name" /proc/cpuinfo | head -1 > $R/host_cpu.txt
for f in $R/bench_*.json; do echo "$f $(cut -c1-200 $f)"; done
exit 0
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_pages4k -o pages4k -- python bench.py --cpu-seconds 0 > $R/prof_pages4k.log 2>&1 || exit 1
for w in pages8k zipf zipf-scattered chunks xxh3-pages4k xxh3-zipf xxh3-chunks xxh3-chained sqlite-verify diskqueue-verify sqlite-seal diskqueue-seal packets-verify redwood-verify redwood-seal; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$w -o $w -- python bench.py --workload $w --steps 20 --cpu-seconds 0 --no-verify > $R/prof_$w.log 2>&1 || exit 1
done
echo rocprof done
[ "${PMC:-1}" = 1 ] || exit 0  # (PMC=0: kernel traces only)
for MODE in pages4k pages8k xxh3 zipf chunks xchunks xzipf scattered; do
  for spec in "fetch FETCH_SIZE" "write WRITE_SIZE" "sq GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
    set -- $spec; name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $P/$MODE -o ${name}_$MODE -- python tools/pmc_probe.py $MODE > $P/$MODE.log 2>&1 || exit 1
  done
done
echo pmc done
