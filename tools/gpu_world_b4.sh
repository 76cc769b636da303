# BVH4 world build (lib_b4): the world GPU tests through it, then the A/B of
# lib (BVH2) vs lib_b4 on the globe (tools/world_bench.py, node visits per
# segment from its counts pass), builds alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
RTW_LIB_PATH=$P/lib_b4/librtw_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_world_b4.log 2>&1 &&
for r in 1 2 3; do
  for L in lib lib_b4; do
    echo "lib $L" >> gpurun_out/wlib_ab.log
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/world_bench.py 7 >> gpurun_out/wlib_ab.log 2>&1 || exit 1
  done
done
