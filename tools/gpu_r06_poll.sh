#!/bin/bash
# Round 6: the wavefront engine's live-count poll.  (1) lib_m (-DRTW_MEASURE)
# with RTW_WF_POLL_CHECK=1: wf_step's published count against wf_count's, per
# batch (mismatches on stderr); (2) lib_m in-process A/B of the published
# count against the wf_count + copy poll (RTW_WF_POLL_KERNEL=1); (3) lib
# against lib_prev (the library before the in-kernel publish), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
OUT=gpurun_out/r06_poll.txt
: > $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "wavefront or wf_" tests \
  > gpurun_out/r06_wf_tests.txt 2>&1 || { tail -30 gpurun_out/r06_wf_tests.txt; exit 1; }
tail -1 gpurun_out/r06_wf_tests.txt >> $OUT
RTW_LIB_PATH=$P/lib_m/librtw_hip.so RTW_WF_POLL_CHECK=1 timeout -k 10 200 python tools/wf_bench.py 1 \
  > gpurun_out/poll_check.out 2> gpurun_out/poll_check.err || exit 1
echo "poll check: $(grep -c 'rtw wf poll' gpurun_out/poll_check.err) mismatching batches" >> $OUT
grep 'rtw wf poll' gpurun_out/poll_check.err | sed -n 1,20p >> $OUT
RTW_LIB_PATH=$P/lib_m/librtw_hip.so timeout -k 10 300 python tools/wf_bench.py 3 - RTW_WF_POLL_KERNEL=1 >> $OUT || exit 1
cat $OUT
TESTS=0 ENGINES=wf ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-lib_prev lib}" bash tools/gpu_r06_ab.sh
