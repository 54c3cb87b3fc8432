# development: rocprofv3 kernel stats of zipf/chunks under pinned routes and block-route thresholds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pr
for cfg in ${CFGS:-"1:4096" "0:4096" "0:8192"}; do
  r=${cfg%%:*}; b=${cfg##*:}
  for w in ${WORKLOADS:-zipf}; do
    d=gpurun_out/pr/${w}_r${r}_b${b}
    FDBCRC_ROUTE=$r FDBCRC_BIGMIN=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o k -- python bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 --no-verify > $d.log 2>&1 || exit 1
    echo "== $w route=$r bigmin=$b"
    cut -d, -f1-4 $d/k_kernel_stats.csv | head -6
  done
done
