#!/bin/bash
# Round 6: the wavefront kernels with the megakernel's closest-hit / scatter
# variant bits (lib_wc: RTW_WF_VAR_EXTRA=kVarCluster; lib_wcs: + RTW_WF_SCATTER_VAR
# = kVarFastSqrt | kVarR0Table): the wavefront GPU tests through lib_wcs, then
# tools/gpu_r06_ab.sh's wavefront A/B against lib.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
for L in ${TEST_LIBS:-lib_wcs}; do
  RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    -m gpu -k "wavefront or wf_" tests > gpurun_out/r06_wfvar_tests_$L.txt 2>&1 || { tail -30 gpurun_out/r06_wfvar_tests_$L.txt; exit 1; }
  echo "$L: $(tail -1 gpurun_out/r06_wfvar_tests_$L.txt)"
done
TESTS=0 ENGINES=wf ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-lib lib_wc lib_wcs}" bash tools/gpu_r06_ab.sh
