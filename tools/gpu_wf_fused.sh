# Fused wavefront engine: wavefront GPU tests (fused / split x both drains),
# the A/B fused vs split (tools/wf_bench.py), rocprofv3 kernel statistics of
# each form, and the fused form's PMC traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_wf.log 2>&1 &&
for r in 1 2 3; do
  for F in 1 0; do
    echo -n "fused=$F " >> gpurun_out/wf_fused_ab.txt
    RTW_WF_FUSED=$F timeout -k 10 200 python tools/wf_bench.py 3 2>/dev/null >> gpurun_out/wf_fused_ab.txt || exit 1
  done
done &&
for F in 1 0; do
  RTW_WF_FUSED=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/wfprof_f$F -o run -- python tools/wf_bench.py 1 > gpurun_out/wfprof_f$F.log 2>&1 || exit 1
done &&
bash tools/gpu_pmc_wf.sh
