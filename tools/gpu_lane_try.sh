# Per-lane BVH traversal trial: the world GPU tests (both traversals) on the product
# library, then world_bench.py on the globe: the union walk and the per-lane walk at two
# register budgets (3 interleaved rounds), and (RTW_MEASURE library lib_m) the per-lane
# walk's yield threshold RTW_WORLD_YIELD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_world.py \
  > gpurun_out/lane_world_tests.txt 2>&1; tail -3 gpurun_out/lane_world_tests.txt
grep -E "globe 1200x675x100|prim tests bvh" gpurun_out/lane_world_tests.txt | cut -c1-200
for r in 1 2 3; do
  timeout -k 10 300 python tools/world_bench.py 7 world_traversal=union world_traversal=lane world_traversal=lane,world_waves=3 2>&1 | sed "s/^/round $r /" | tee -a gpurun_out/lane_try.txt
done
for y in 12 16 24 32; do
  RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_m/librtw_hip.so RTW_WORLD_YIELD=$y timeout -k 10 300 \
    python tools/world_bench.py 7 world_traversal=lane 2>&1 | sed "s/^/yield $y /" | tee -a gpurun_out/lane_try.txt
done
