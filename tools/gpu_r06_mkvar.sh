#!/bin/bash
# Round 6: megakernel variant A/Bs.  The megakernel parity tests
# (tests/test_gpu_parity.py) through each of TEST_LIBS, then tools/gpu_r06_ab.sh's
# megakernel A/B (bench.py configs[1] f64 + f32 lines) over LIBS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
for L in ${TEST_LIBS:-}; do
  RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py > gpurun_out/r06_mkvar_tests_$L.txt 2>&1 || { tail -30 gpurun_out/r06_mkvar_tests_$L.txt; exit 1; }
  echo "$L: $(tail -1 gpurun_out/r06_mkvar_tests_$L.txt)"
done
TESTS=0 ENGINES=mk ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-lib}" bash tools/gpu_r06_ab.sh
