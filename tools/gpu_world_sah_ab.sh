# World BVH builder SAH-cost A/B (globe): world GPU tests under a variant tree, then tools/world_ab.py over RTW_SAH_W values.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
# (the RTW_SAH_W builder knob was removed after this A/B: profiles/r02/world_sah_cost_ab.txt)
RTW_SAH_W=-1.5 timeout -k 10 300 python -u -m pytest tests/test_gpu_world.py -x -q --timeout 200 > gpurun_out/pytest_world_sah.log 2>&1 &&
timeout -k 10 400 python tools/world_ab.py 7 'RTW_SAH_W=0;RTW_SAH_W=-0.75;RTW_SAH_W=-1.25;RTW_SAH_W=-1.5' 2 > gpurun_out/sah_ab.log 2>&1
