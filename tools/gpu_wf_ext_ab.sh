# wf_extend instantiation A/B: builds in LIBS (RTW_LIB_PATH), alternated in
# separate processes, after the wavefront GPU tests; then rocprofv3 kernel
# statistics of one wavefront frame for each build (per-kernel averages).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
LIBS=${LIBS:-lib lib_c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 300 > gpurun_out/pytest_wf.log 2>&1 &&
for r in 1 2 3; do
  for L in $LIBS; do
    echo -n "$L " >> gpurun_out/wf_ab.log
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/wf_bench.py 3 2>/dev/null >> gpurun_out/wf_ab.log || exit 1
  done
done
for L in $LIBS; do
  RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/wfprof_$L -o run -- python tools/wf_bench.py 1 > gpurun_out/wfprof_$L.log 2>&1 || exit 1
done
