# HBM traffic of the wavefront engine's bounce kernels (BASELINE configs[3]):
# FETCH_SIZE and WRITE_SIZE in separate PMC passes over one f64 frame; then
# two issue passes (VALU / SALU / LDS instructions, busy and wait cycles).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_fetch -o run \
  --pmc FETCH_SIZE -- python tools/prof_run.py wf64 > gpurun_out/wf_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_write -o run \
  --pmc WRITE_SIZE -- python tools/prof_run.py wf64 > gpurun_out/wf_write.log 2>&1 &&
python tools/wf_traffic_json.py gpurun_out/wf_fetch gpurun_out/wf_write gpurun_out/wf_traffic.json &&
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_issue_a -o run \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM \
  -- python tools/prof_run.py wf64 > gpurun_out/wf_issue_a.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_issue_b -o run \
  --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS \
  -- python tools/prof_run.py wf64 > gpurun_out/wf_issue_b.log 2>&1
