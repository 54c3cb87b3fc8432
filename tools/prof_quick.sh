# development: rocprofv3 kernel stats of a few bench workloads (WORKLOADS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pq
for w in ${WORKLOADS:-chunks}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pq/$w -o $w -- python bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 --no-verify > gpurun_out/pq/$w.log 2>&1 || exit 1
  cut -d, -f1-4 gpurun_out/pq/$w/${w}_kernel_stats.csv | head -8
done
