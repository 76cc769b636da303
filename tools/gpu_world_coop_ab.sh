# World kernel: GPU world tests, then cooperative vs per-lane unit-ball
# sampling (RTW_WORLD_OCC 4 vs 14) and the previous build (lib_c), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -x -q --timeout 300 > gpurun_out/pytest_world.log 2>&1 &&
for r in 1 2; do
  for cfg in "lib 4" "lib 14" "lib_c 4"; do
    set -- $cfg
    echo "lib $1 occ $2" >> gpurun_out/wcoop_ab.log
    RTW_WORLD_OCC=$2 RTW_LIB_PATH=$P/$1/librtw_hip.so timeout -k 10 200 python tools/world_bench.py 6,7 >> gpurun_out/wcoop_ab.log 2>&1 || exit 1
  done
done
