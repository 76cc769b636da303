# Wavefront engine bring-up: its GPU parity tests, the megakernel parity tests
# (after the rtw_device.hpp refactor), then the bench line (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_wavefront.py -x -q -s > gpurun_out/pytest_wf.log 2>&1 &&
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err
