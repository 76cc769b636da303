set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py tests/test_capi_cpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/wf_finish_tests.log 2>&1 &&
bash tools/gpu_pmc_wf.sh &&
timeout -k 10 300 python bench.py --engine wavefront --no-cpu-baseline --no-f32-variant --no-world-variants \
  --steps 5 --warmup 2 > gpurun_out/wf_head.json 2> gpurun_out/wf_head.err
