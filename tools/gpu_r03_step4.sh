# Survivor compaction (kVarCompact, lib_cmp): the megakernel parity tests on
# lib_cmp, timing A/B lib vs lib_cmp, VALU PMC pass of lib_cmp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_cmp/librtw_hip.so \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_cmp.log 2>&1 &&
ENGINE=mk LIBS="lib lib_cmp" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null 2>&1 &&
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_cmp/librtw_hip.so TAG=r03c bash tools/gpu_pmc_valu.sh
