# World kernel A/B of two builds (lib vs lib_c, RTW_LIB_PATH) after the GPU
# world tests, alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -x -q --timeout 300 > gpurun_out/pytest_world.log 2>&1 &&
for r in 1 2 3; do
  for L in ${LIBS:-lib lib_c}; do
    echo "lib $L" >> gpurun_out/wlib_ab.log
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/world_bench.py ${SCENES:-7,6} >> gpurun_out/wlib_ab.log 2>&1 || exit 1
  done
done
