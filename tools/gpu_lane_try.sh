# Per-lane BVH traversal trial: the world GPU tests (both traversals) on the product
# library, then world_bench.py on the globe and scene 1: the union walk and the
# per-lane walk at two register budgets, and (RTW_MEASURE library lib_m) the
# per-lane walk's yield threshold RTW_WORLD_YIELD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_world.py \
  > gpurun_out/lane_world_tests.txt 2>&1; tail -3 gpurun_out/lane_world_tests.txt
grep -E "globe 1200x675x100|prim tests bvh" gpurun_out/lane_world_tests.txt | cut -c1-200
timeout -k 10 300 python tools/world_bench.py 7,1 - world_traversal=lane world_traversal=lane,world_waves=3 2>&1 | tee gpurun_out/lane_try.txt
for y in 0 16 24 32 40; do
  RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_m/librtw_hip.so RTW_WORLD_YIELD=$y timeout -k 10 300 \
    python tools/world_bench.py 7 world_traversal=lane world_traversal=lane,world_waves=3 2>&1 | sed "s/^/yield $y /" | tee -a gpurun_out/lane_try.txt
done
# wavefront: bounce segments per wf_step launch (RTW_WF_BOUNCES, RTW_MEASURE library):
# bit identity of 2 bounces per launch (the wavefront parity tests), then timing
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_m/librtw_hip.so RTW_WF_BOUNCES=2 timeout -k 10 400 \
  python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wavefront.py \
  -k "fused and (config2 or parity or exactly_once)" > gpurun_out/wf_bounces_tests.txt 2>&1; tail -2 gpurun_out/wf_bounces_tests.txt
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_m/librtw_hip.so timeout -k 10 300 \
  python tools/wf_bench.py 3 - RTW_WF_BOUNCES=2 RTW_WF_BOUNCES=3 RTW_WF_BOUNCES=4 2>&1 | tee gpurun_out/wf_bounces.txt
