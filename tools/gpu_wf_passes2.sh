set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60 RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_m/librtw_hip.so
timeout -k 10 500 python tools/wf_bench.py 4 RTW_WF_PASSES=8 RTW_WF_PASSES=12 RTW_WF_PASSES=16 RTW_WF_PASSES=8,sets=1 RTW_WF_PASSES=8,sets=3 RTW_WF_PASSES=8,paths=1048576 RTW_WF_PASSES=8,paths=524288 RTW_WF_PASSES=16,sets=1 \
  > gpurun_out/wf_passes_ab2.txt 2>&1; r=$?; cat gpurun_out/wf_passes_ab2.txt; exit $r
