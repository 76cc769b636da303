# World-kernel iteration: GPU world + cover parity tests, then world timings
# at each register budget (scenes 6 Cornell, 7 globe, 1 cover, 3 Perlin).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py tests/test_gpu_parity.py -x -q --timeout 300 \
  > gpurun_out/pytest_world.log 2>&1 &&
bash tools/gpu_world_ab.sh
