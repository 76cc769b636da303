# Survivor-loop cost by phase duplication: timing A/B lib vs lib_dup (the
# clustered survivors' exact tests run twice) + the VALU PMC pass of lib_dup.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ENGINE=mk LIBS="lib lib_dup" ROUNDS=2 bash tools/gpu_ab.sh > /dev/null 2>&1 &&
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_dup/librtw_hip.so TAG=r03d bash tools/gpu_pmc_valu.sh
