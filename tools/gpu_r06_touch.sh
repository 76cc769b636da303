#!/bin/bash
# Round 6: the per-lane walk also touching record ref + 1 with each node visit (lib_lt,
# -DRTW_LANE_TOUCH=1) vs lib: the world GPU tests through lib_lt, then the world A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_lt/librtw_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_world.py > gpurun_out/r06_touch_tests.txt 2>&1 || { tail -30 gpurun_out/r06_touch_tests.txt; exit 1; }
tail -1 gpurun_out/r06_touch_tests.txt
TESTS=0 ENGINES=world SCENES=7 ROUNDS=${ROUNDS:-5} LIBS="lib lib_lt" bash tools/gpu_r06_ab.sh
