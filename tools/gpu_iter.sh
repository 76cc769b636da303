# Iteration loop: GPU parity tests + bench (no CPU baseline) + phase profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1
