# Choosing the trace-kernel defaults: device math check, parity tests, and a
# longer interleaved A/B of the candidate variants in each precision.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_math.py tests/test_gpu_parity.py -x -q --timeout 200 \
  > gpurun_out/pytest_ab.log 2>&1 &&
timeout -k 10 400 python tools/ab_variants.py f64 ${VARS64:-4,516,33284,164356} 8 > gpurun_out/ab_f64.log 2>&1 &&
timeout -k 10 400 python tools/ab_variants.py f32 ${VARS32:-8,520,131592} 8 > gpurun_out/ab_f32.log 2>&1
