# wf_finish (drain in registers) vs the queue drain: wavefront GPU tests with
# both drains, then the configs[1] wavefront frame timed each way.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/wf_finish_tests.log 2>&1 &&
for f in 0 1 0 1; do
  RTW_WF_FINISH=$f timeout -k 10 300 python bench.py --engine wavefront --no-cpu-baseline --no-f32-variant \
    --no-world-variants --steps 5 --warmup 2 > gpurun_out/wf_finish_$f.json 2>> gpurun_out/wf_finish_ab.err || exit $?
  echo "RTW_WF_FINISH=$f $(python -c "import json;d=json.load(open('gpurun_out/wf_finish_$f.json'));print(d['value'],d['ms_per_step'],d['roofline']['loop_ms_per_frame'])")" >> gpurun_out/wf_finish_ab.txt
done
