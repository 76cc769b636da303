# RCCL one-rank rehearsal test + world-kernel OCC 4 vs 5 A/B (globe, Cornell).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rccl.py > gpurun_out/rccl.log 2>&1 &&
timeout -k 10 400 python tools/world_ab.py 7,6 'RTW_WORLD_OCC=4;RTW_WORLD_OCC=5' 2 > gpurun_out/world_occ5_ab.txt 2>&1
