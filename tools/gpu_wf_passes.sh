# Queue passes per wf_step launch (RTW_WF_PASSES, -DRTW_MEASURE library lib_m):
# bit identity against the megakernel, then the configs[1] wavefront frame
# (tools/wf_bench.py, interleaved) at 1 / 2 / 3 / 4 passes and K = 2 bounces;
# then the 2-rank gloo rehearsal with 10 timed steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
export RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_m/librtw_hip.so
timeout -k 10 300 python tools/wf_passes_check.py - RTW_WF_PASSES=2 RTW_WF_PASSES=3 RTW_WF_PASSES=4 \
  RTW_WF_PASSES=2,bounces=2 RTW_WF_PASSES=3,sets=1 RTW_WF_PASSES=2,drain=slots RTW_WF_PASSES=2,drain=none \
  > gpurun_out/wf_passes_check.txt 2>&1; r=$?; cat gpurun_out/wf_passes_check.txt; [ $r -eq 0 ] &&
timeout -k 10 400 python tools/wf_bench.py 4 - RTW_WF_PASSES=2 RTW_WF_PASSES=3 RTW_WF_PASSES=4 RTW_WF_PASSES=8 bounces=2 \
  > gpurun_out/wf_passes_ab.txt 2>&1 && cat gpurun_out/wf_passes_ab.txt &&
unset RTW_LIB_PATH &&
RTW_DIST_BACKEND=gloo RTW_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 \
  --no-cpu-baseline --no-wavefront-variant --no-world-variants --no-f32-variant \
  > gpurun_out/dist_rehearsal10.json 2> gpurun_out/dist_rehearsal10.err && tail -c 600 gpurun_out/dist_rehearsal10.json
