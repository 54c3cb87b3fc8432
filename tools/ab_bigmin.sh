# development: varlen probes and bench lines at several block-route thresholds ($BIGMINS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for b in ${BIGMINS:-0 4096 16384}; do
  echo "== FDBCRC_BIGMIN=$b"
  FDBCRC_BIGMIN=$b timeout -k 10 300 python tools/probe_varlen.py $CASES 2>&1 | grep -v amdgpu.ids || exit 1
done
