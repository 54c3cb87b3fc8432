# development: rocprofv3 kernel stats of probe_varlen.py cases ($CASES)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
timeout -k 10 300 python tools/probe_varlen.py $CASES 2>&1 | tee gpurun_out/pp/probe.txt || exit 1
for c in $CASES; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp/$c -o k -- python tools/probe_varlen.py "$c" > gpurun_out/pp/$c.log 2>&1 || exit 1
  echo "== $c"; cut -d, -f1-4 gpurun_out/pp/$c/k_kernel_stats.csv | grep -v splitmix | head -8
done
