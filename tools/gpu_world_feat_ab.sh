# World kernel feature-set instantiations: GPU tests (bit identity across
# budgets and feature sets) + A/B of feature set x occupancy on the globe and Cornell.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_world.log 2>&1 &&
timeout -k 10 400 python tools/world_ab.py 7,6 \
  'RTW_WORLD_FEAT=all,RTW_WORLD_OCC=4;RTW_WORLD_FEAT=,RTW_WORLD_OCC=4;RTW_WORLD_FEAT=,RTW_WORLD_OCC=3' 2 \
  > gpurun_out/world_feat_ab.txt 2> gpurun_out/world_feat_ab.err
