#!/bin/bash
# Round 6: the per-lane walk's LDS node cache (the top kNodeCache records,
# breadth-first).  The world GPU tests through lib, then the world A/B of
# lib_base (the library before it) against lib (tools/gpu_r06_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_world.py \
  > gpurun_out/r06_ncache_tests.txt 2>&1 || { tail -30 gpurun_out/r06_ncache_tests.txt; exit 1; }
tail -1 gpurun_out/r06_ncache_tests.txt
TESTS=0 ENGINES=world ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-lib_base lib}" bash tools/gpu_r06_ab.sh
