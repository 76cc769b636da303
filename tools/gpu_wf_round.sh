# Wavefront engine evidence with the queue sets (round 4): the wavefront GPU
# tests, a kernel trace of one frame (overlap of the sets' launches,
# tools/wf_overlap_summary.py), the HBM / issue PMC passes (tools/gpu_pmc_wf.sh)
# and an in-process A/B of 1 vs 2 sets (tools/wf_bench.py).  Round 5 moved the set count into
# rtw_params.wf_sets (the library reads no RTW_WF_SETS): the configurations name the field.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wavefront.py \
    > gpurun_out/wf_tests.txt 2>&1 || { tail -30 gpurun_out/wf_tests.txt; exit 1; }
  tail -2 gpurun_out/wf_tests.txt
fi
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_trace -o run \
  -- python tools/prof_run.py wf64 > gpurun_out/wf_trace.log 2>&1 &&
python tools/wf_overlap_summary.py gpurun_out/wf_trace/run_kernel_trace.csv gpurun_out/wf_overlap.json &&
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_trace1 -o run \
  -- python tools/prof_run.py wf64 1 wf_sets=1 > gpurun_out/wf_trace1.log 2>&1 &&
python tools/wf_overlap_summary.py gpurun_out/wf_trace1/run_kernel_trace.csv gpurun_out/wf_overlap_sets1.json &&
bash tools/gpu_pmc_wf.sh && python tools/wf_kernel_pmc.py gpurun_out/wf_issue_a gpurun_out/wf_issue_b > gpurun_out/wf_issue.txt &&
timeout -k 10 300 python -u tools/wf_bench.py 5 sets=1 sets=2 "sets=1,paths=1048576" > gpurun_out/wf_sets_final_ab.txt 2>&1 &&
cat gpurun_out/wf_issue.txt gpurun_out/wf_sets_final_ab.txt | grep -v amdgpu.ids
