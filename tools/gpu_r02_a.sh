# After the drain check / globe asset changes: world + wavefront GPU tests,
# then the world-kernel timings and PMC passes (tools/gpu_r02_world.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py tests/test_gpu_wavefront.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_world_wf.log 2>&1 &&
bash tools/gpu_r02_world.sh
