# World traversal with fields re-read from the kernel argument (lib_kw) vs SGPR copy (lib): world GPU
# tests through lib_kw, then the globe A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
RTW_LIB_PATH=$P/lib_kw/librtw_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_world_kw.log 2>&1 &&
for r in 1 2 3; do
  for L in lib lib_kw; do
    echo "conf $L" >> gpurun_out/wlib_kw.log
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/world_bench.py 7,6 >> gpurun_out/wlib_kw.log 2>&1 || exit 1
  done
done
