# Wavefront polled batches of one 8-pass launch (lib) vs two (lib_pv): the drain starts up to a batch earlier.
# Wavefront GPU tests through lib first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/iters_wf_tests.txt 2>&1; r=$?; tail -2 gpurun_out/iters_wf_tests.txt; [ $r -eq 0 ] &&
rm -f gpurun_out/ab_wf.txt &&
ENGINE=wf LIBS="lib lib_pv" ROUNDS=4 bash tools/gpu_ab.sh > /dev/null && cat gpurun_out/ab_wf.txt
