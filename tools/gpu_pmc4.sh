# VALU / SALU instruction counts and wait cycles of the default variants vs
# RTW_VARIANT=$ALT (A/B of instruction mix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
P=tools/prof_run.py
run() { name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_$name -o run --pmc "$@" \
    -- python $P both > gpurun_out/pmc_$name.log 2>&1; }
CNT="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"
run def $CNT &&
RTW_VARIANT=${ALT64:-68} run alt64 $CNT &&
RTW_VARIANT=${ALT32:-72} run alt32 $CNT
