set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in ${ROUTES:-0 1 2}; do
  echo "== FDBCRC_ROUTE=$r"
  FDBCRC_ROUTE=$r timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "${K:-route or random_varlen or chunk or configs}" --timeout 120 --timeout-method thread > gpurun_out/routes_$r.txt 2>&1
  grep -E "AssertionError|passed|failed" gpurun_out/routes_$r.txt | cut -c1-600
done
