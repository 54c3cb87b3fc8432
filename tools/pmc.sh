# rocprofv3 counter passes for the page kernel (run on the GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/pmc
mkdir -p $P
run() { # name counters... ; mode from $MODE
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $P/$MODE -o $1_$MODE -- python tools/pmc_probe.py $MODE > $P/$MODE.log 2>&1
}
for MODE in pages4k stride0; do
  run fetch FETCH_SIZE || exit $?
  run write WRITE_SIZE || exit $?
  run sq GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES || exit $?
  run sq2 GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD || exit $?
done
ls -R $P | head -50
