# Wavefront queue sets (RTW_WF_SETS): in-process A/B of set counts, queue
# sizes and per-set grids (tools/wf_bench.py), then the wavefront GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
CFGS=${CFGS:-"RTW_WF_SETS=1 RTW_WF_SETS=2 RTW_WF_SETS=2,paths=2097152 RTW_WF_SETS=3,paths=1572864 RTW_WF_SETS=4,paths=2097152 RTW_WF_SETS=2,RTW_WF_SET_GRID=2 RTW_WF_SETS=2,paths=2097152,RTW_WF_SET_GRID=2"}
timeout -k 10 400 python -u tools/wf_bench.py ${N:-3} $CFGS > gpurun_out/wf_sets_ab.txt 2>&1 && cat gpurun_out/wf_sets_ab.txt || exit 1
if [ -n "${TESTS:-1}" ] && [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wavefront.py \
    > gpurun_out/wf_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/wf_tests.txt; exit $rc
fi
