# Evidence for one bench line on a GPU box: the line with its CPU baseline,
# then its rocprofv3 kernel stats (outputs under gpurun_out/$ROUND/, copied
# into profiles/$ROUND/ afterwards).   WL=<workload> ROUND=round6 bash tools/evidence_line.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=gpurun_out/${ROUND:-round6}
mkdir -p $R
for w in $WL; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --cpu-seconds 5 > $R/bench_$w.json 2> $R/bench_$w.err || { tail -3 $R/bench_$w.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof_$w -o $w -- python bench.py --workload $w --steps 20 --cpu-seconds 0 --no-verify > $R/prof_$w.log 2>&1 || exit 1
  cut -c1-300 $R/bench_$w.json
done
