# Megakernel change: GPU parity tests on the current build, then the A/B of
# lib (current) vs LIBS' other builds (tools/gpu_mk_conf_ab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_parity.log 2>&1 &&
CONFS="${CONFS:-lib lib_old}" bash tools/gpu_mk_conf_ab.sh
