# Per-lane BVH traversal trial: the world GPU tests (both traversals), then
# world_bench.py on the globe and scene 1 with the union walk and the per-lane
# walk at several register budgets (rtw_params fields, in-process).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_world.py \
  > gpurun_out/lane_world_tests.txt 2>&1; tail -3 gpurun_out/lane_world_tests.txt; grep -E "lane|union" gpurun_out/lane_world_tests.txt | grep -v PASSED | head -20
timeout -k 10 300 python tools/world_bench.py 7,1 - world_traversal=lane world_traversal=lane,world_waves=3 2>&1 | tee gpurun_out/lane_try.txt
