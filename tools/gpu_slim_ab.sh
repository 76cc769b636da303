# Per-lane walk loads: slim (sphere centre / r^2 / meta 64 B, moving fields only for kind 1; the
# node's refs without its padding: lib) vs full records (lib_fr, -DRTW_LANE_FULL_REC), each with
# the 4-wide (lane) and binary (lane2) BVH; world GPU tests through lib first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/slim_world_tests.txt 2>&1; r=$?; tail -2 gpurun_out/slim_world_tests.txt; [ $r -eq 0 ] &&
for k in 1 2 3 4; do
  for L in lib lib_fr; do
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 300 python tools/world_bench.py 7 world_traversal=lane world_traversal=lane2 \
      2>&1 | grep -v amdgpu.ids | sed -E 's/"W": .*"linear": false, //' | cut -c1-170 | sed "s/^/$L round $k /" || exit 1
  done
done
