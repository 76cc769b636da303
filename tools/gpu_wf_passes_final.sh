# Queue passes per launch in the product library: the wavefront GPU tests, the
# wavefront PMC passes (traffic + issue), then the bench line without the
# world / f32 variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out/evp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/evp/pytest_wavefront.txt 2>&1; r=$?; tail -3 gpurun_out/evp/pytest_wavefront.txt; [ $r -eq 0 ] &&
bash tools/gpu_pmc_wf.sh > /dev/null && cp gpurun_out/wf_traffic.json gpurun_out/evp/ &&
python tools/wf_kernel_pmc.py gpurun_out/wf_issue_a gpurun_out/wf_issue_b > gpurun_out/evp/wf_issue.txt &&
cp gpurun_out/evp/wf_traffic.json profiles/r05/ &&
timeout -k 10 600 python bench.py --no-world-variants --no-f32-variant --no-cpu-baseline > gpurun_out/evp/bench_wf.json 2> gpurun_out/evp/bench_wf.err &&
python -c "import json; d=json.load(open('gpurun_out/evp/bench_wf.json')); w=d['wavefront_variant']; print(d['value'], w['value'], w['roofline']['frac'], w['roofline']['traffic'], w['bounces_per_launch'])"
