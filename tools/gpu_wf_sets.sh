# Wavefront queue sets (rtw_params.wf_sets: "sets=N" in tools/wf_bench.py; the
# library reads no RTW_WF_SETS since round 5): in-process A/B of set counts, queue
# sizes and per-set grids (RTW_WF_SET_GRID: a development knob, -DRTW_MEASURE
# library only), then the wavefront GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
CFGS=${CFGS:-"sets=1 sets=2 sets=2,paths=2097152 sets=3,paths=1572864 sets=4,paths=2097152 sets=2,RTW_WF_SET_GRID=2 sets=2,paths=2097152,RTW_WF_SET_GRID=2"}
timeout -k 10 400 python -u tools/wf_bench.py ${N:-3} $CFGS > gpurun_out/wf_sets_ab.txt 2>&1 && cat gpurun_out/wf_sets_ab.txt || exit 1
if [ -n "${TESTS:-1}" ] && [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wavefront.py \
    > gpurun_out/wf_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/wf_tests.txt; exit $rc
fi
