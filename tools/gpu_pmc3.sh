# Phase stamps + VALU utilisation / instruction mix of the default variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
P=tools/prof_run.py
run() { name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$name -o run --pmc "$@" \
    -- python $P both > gpurun_out/pmc_$name.log 2>&1; }
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1 &&
run util SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES &&
run mix SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_LDS
