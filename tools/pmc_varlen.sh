set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest.txt 2>&1; tail -1 gpurun_out/pytest.txt; grep -q passed gpurun_out/pytest.txt && ! grep -q failed gpurun_out/pytest.txt || exit 1
P=gpurun_out/pmc3
mkdir -p $P
for MODE in chunks zipf pages4k; do
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-trace --output-format csv -d $P/$MODE -o sq_$MODE -- python tools/pmc_probe.py $MODE > $P/$MODE.log 2>&1 || exit 1
done
echo ok
