# World kernel check: its GPU tests (BVH == linear == Tier B), then the
# globe and Cornell lines of tools/world_bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -x -q --timeout 300 > gpurun_out/pytest_world.log 2>&1 &&
timeout -k 10 300 python tools/world_bench.py 7,6 > gpurun_out/world_check.log 2>&1
