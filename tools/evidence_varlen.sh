# Bench lines + rocprofv3 kernel stats for the varlen workloads (GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=gpurun_out/varlen
mkdir -p $R
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.txt 2>&1 || exit 1
for w in zipf chunks; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --cpu-seconds 5 > $R/bench_$w.json 2> $R/bench_$w.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$w -o $w -- python bench.py --workload $w --steps 20 --cpu-seconds 0 > $R/prof_$w.log 2>&1 || exit 1
done
cat $R/bench_*.json | cut -c1-200
