# World kernel with the fast exact f64 sqrt and Markstein normalise (lib)
# vs the previous build (lib_o): GPU world tests on lib, then the A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -x -q --timeout 300 > gpurun_out/pytest_world_sqrt.log 2>&1 &&
for r in 1 2 3; do
  for L in lib_o lib; do
    echo "lib $L" >> gpurun_out/wsqrt_ab.log
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/world_bench.py 7,6 >> gpurun_out/wsqrt_ab.log 2>&1 || exit 1
  done
done
