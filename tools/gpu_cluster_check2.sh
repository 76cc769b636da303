# Clustered pretest build lib_k: GPU parity tests through it, its kernel
# counts (cluster skip rate), then the megakernel A/B lib vs lib_k.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
RTW_LIB_PATH=$P/lib_k/librtw_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wavefront.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_k.log 2>&1 &&
RTW_LIB_PATH=$P/lib_k/librtw_hip.so bash tools/gpu_counts.sh &&
CONFS="lib lib_k" bash tools/gpu_mk_conf_ab.sh
