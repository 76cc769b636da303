# VALU issue accounting of ONE f64 trace launch (configs[1]): counter list +
# per-dispatch PMC passes (each pass its own run, <= 8 SQ counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01v}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_a -o run \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
  -- python tools/prof_run.py f64 > gpurun_out/${TAG}_a.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_b -o run \
  --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH \
  -- python tools/prof_run.py f64 > gpurun_out/${TAG}_b.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_c -o run \
  --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  -- python tools/prof_run.py f64 > gpurun_out/${TAG}_c.log 2>&1
