# Clustered pretest (kVarCluster) build lib_k: GPU parity tests through it,
# then the megakernel A/B lib vs lib_k (tools/gpu_mk_lib_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
RTW_LIB_PATH=$P/lib_k/librtw_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_k.log 2>&1 &&
LIBS="lib lib_k" bash tools/gpu_mk_lib_ab.sh
