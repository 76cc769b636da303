# Round 3: lane home block in LDS (lib_home, trace VAR kVarHomeLds): parity
# tests + timing A/B against lib; wavefront queue-size / grid sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ENGINE=mk LIBS="lib lib_home" TESTS="tests/test_gpu_parity.py" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null 2>&1 &&
timeout -k 10 600 python tools/wf_bench.py 2 - paths=983040 paths=1310720 paths=1638400 paths=2097152 RTW_WF_GRID=4 \
  paths=1310720,RTW_WF_GRID=4 > gpurun_out/wf_sweep.txt 2>&1
