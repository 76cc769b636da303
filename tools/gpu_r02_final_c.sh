# Round-2 evidence after the world kernel's register-held stack top: every GPU
# test + smoke(), the world-kernel PMC passes on the globe (configs[4]), then
# the bench line and its rocprofv3 kernel statistics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
SCENE=7 bash tools/gpu_world_pmc.sh &&
bash tools/gpu_r02_bench.sh
