# SQ counter passes (development): per-unit instruction mix and wait cycles
# for the page kernel and the varlen engine.  MODES="pages4k v4096 ..." bash tools/pmc_sq.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/pmcsq
mkdir -p $P
for MODE in ${MODES:-pages4k v4096 v1024 zipf}; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $P/$MODE -o a_$MODE -- python tools/pmc_probe.py $MODE > $P/$MODE.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $P/$MODE -o b_$MODE -- python tools/pmc_probe.py $MODE >> $P/$MODE.log 2>&1 || exit 1
done
echo ok
