# Per-lane BVH traversal build (lib_c, -DRTW_WORLD_LANE_TRAV=1): GPU world
# parity tests on it, then globe timing vs the default build (OCC 4 and 3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
RTW_LIB_PATH=$P/lib_c/librtw_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -x -q --timeout 300 > gpurun_out/pytest_world_lane.log 2>&1 &&
for r in 1 2; do
  for C in "lib 4" "lib_c 4" "lib_c 3"; do
    set -- $C
    echo "lib $1 occ $2" >> gpurun_out/wlane_ab.log
    RTW_WORLD_OCC=$2 RTW_LIB_PATH=$P/$1/librtw_hip.so timeout -k 10 200 python tools/world_bench.py 7 >> gpurun_out/wlane_ab.log 2>&1 || exit 1
  done
done
