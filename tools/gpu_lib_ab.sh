# A/B of whole library builds (RTW_LIB_PATH) on the world scenes: rounds of
# lib, lib_b, lib_c alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
for r in 1 2; do
  for L in lib lib_b lib_c; do
    echo "lib $L" >> gpurun_out/lib_ab.log
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/world_bench.py ${SCENES:-6,7} >> gpurun_out/lib_ab.log 2>&1 || exit 1
  done
done
