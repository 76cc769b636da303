# Wavefront iteration check: its GPU tests, then the configs[1] frame at the
# default capacity (f64, f32), twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/wf_iter_tests.log 2>&1 &&
timeout -k 10 300 python tools/wf_sweep.py f64,f32 1048576 > gpurun_out/wf_iter.txt 2>&1 &&
timeout -k 10 300 python tools/wf_sweep.py f64,f32 1048576 >> gpurun_out/wf_iter.txt 2>&1
