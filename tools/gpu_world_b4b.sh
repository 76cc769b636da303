# BVH4 A/B, second version: lib (BVH2) vs lib_b4 at 4 and 3 waves/SIMD on the globe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
RTW_LIB_PATH=$P/lib_b4/librtw_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_world_b4.log 2>&1 &&
for r in 1 2; do
  for C in lib lib_b4 lib_b4+RTW_WORLD_OCC=3; do
    L=${C%%+*}; E=""; [ "$C" != "$L" ] && E=${C#*+}
    echo "conf $C" >> gpurun_out/wlib_ab2.log
    env $E RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/world_bench.py 7 >> gpurun_out/wlib_ab2.log 2>&1 || exit 1
  done
done
