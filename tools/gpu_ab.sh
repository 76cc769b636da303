set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python tools/ab_variants.py f64 ${VARS64:-0,16} 5 > gpurun_out/ab_f64.log 2>&1 &&
timeout -k 10 300 python tools/ab_variants.py f32 ${VARS32:-8,24} 5 > gpurun_out/ab_f32.log 2>&1 &&
if [ -n "$COUNTS" ]; then bash tools/gpu_counts.sh; fi
