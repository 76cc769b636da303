# World kernel after a change: the world GPU tests, then the globe and Cornell timings (3 rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/world_check_tests.txt 2>&1; r=$?; tail -2 gpurun_out/world_check_tests.txt; [ $r -eq 0 ] &&
timeout -k 10 300 python tools/world_bench.py 7,6,1 2>&1 | sed -E 's/"W": .*"linear": false, //' | cut -c1-260
