# Round 3: software-pipelined wf_step (next segment's paths loaded during the
# closest hit): wavefront parity tests through lib_pf4, then the timing A/B of
# lib (5 waves), lib_o4 (4 waves), lib_pf4 (prefetch, 4 waves), lib_pf5
# (prefetch, 5 waves, spills).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
ENGINE=wf LIBS="lib_pf4" TESTS="tests/test_gpu_wavefront.py" ROUNDS=0 bash tools/gpu_ab.sh > /dev/null 2>&1 &&
ENGINE=wf LIBS="lib lib_o4 lib_pf4 lib_pf5" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null 2>&1
