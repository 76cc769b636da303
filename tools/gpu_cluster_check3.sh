# Cluster size A/B: parity through lib_k4 (4-slot clusters), counts of
# lib_k and lib_k4, then the megakernel A/B of lib, lib_k, lib_k4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
RTW_LIB_PATH=$P/lib_k4/librtw_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_k4.log 2>&1 &&
RTW_LIB_PATH=$P/lib_k4/librtw_hip.so bash tools/gpu_counts.sh && mv gpurun_out/counts.log gpurun_out/counts_k4.log &&
RTW_LIB_PATH=$P/lib_k/librtw_hip.so bash tools/gpu_counts.sh && mv gpurun_out/counts.log gpurun_out/counts_k.log &&
CONFS="lib lib_k lib_k4" bash tools/gpu_mk_conf_ab.sh
