# Round 3 checkpoint: every GPU test + smoke on the current build, then the
# A/B of the round-2 build (lib_o) against it (ENGINES, default "mk").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
for e in ${ENGINES:-mk}; do
  ENGINE=$e LIBS="${LIBS:-lib_o lib}" ROUNDS=${ROUNDS:-3} bash tools/gpu_ab.sh > /dev/null 2>&1 || exit 1
done
