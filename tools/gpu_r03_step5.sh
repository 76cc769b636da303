# Round 3: survivor compaction (lib_cmp) and sign-ordered BVH children
# (lib_so, RTW_WORLD_SIGNORDER=1): parity tests through each candidate, then
# timing A/Bs against lib.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ENGINE=mk LIBS="lib lib_cmp" TESTS="tests/test_gpu_parity.py" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null 2>&1 &&
ENGINE=world LIBS="lib lib_so" TESTS="tests/test_gpu_world.py" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null 2>&1
