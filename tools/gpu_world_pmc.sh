# PMC passes over the world kernel (scene $SCENE, one render of main.zig's
# settings; tools/world_prof_run.py): issue / wait breakdown, VALU issue,
# instruction mix, and the HBM traffic (FETCH_SIZE, WRITE_SIZE in separate
# passes, per MI355X_MICROARCH.md), and the vector memory pipeline's busy shares (TA address
# processing, TD data return).  Output: gpurun_out/wpmc_${SCENE}_{a,b,c,f,w,t}.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${SCENE:-7}
CFG=${CFG:--}  # rtw_params fields for tools/world_prof_run.py (e.g. world_traversal=lane)
O=${OUT:-$S}   # output tag: gpurun_out/wpmc_${O}_*
run() {  # $1 = pass tag, rest = counters
  local tag=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wpmc_${O}_$tag -o run \
    --pmc "$@" -- python tools/world_prof_run.py $S 1 $CFG > gpurun_out/wpmc_${O}_$tag.log 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM &&
run b SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS &&
run c SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 &&
run f FETCH_SIZE &&
run w WRITE_SIZE &&
run t GRBM_GUI_ACTIVE TA_BUSY_avr TD_TD_BUSY_sum
