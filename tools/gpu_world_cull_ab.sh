# World kernel leaf pretest: GPU world tests + A/B (pretest on/off) on the globe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_world.log 2>&1 &&
timeout -k 10 400 python tools/world_ab.py 7 'RTW_WORLD_NOCULL=1;RTW_WORLD_NOCULL=' 3 \
  > gpurun_out/world_cull_ab.txt 2> gpurun_out/world_cull_ab.err
