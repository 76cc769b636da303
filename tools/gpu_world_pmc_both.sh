# World-kernel PMC passes of the globe (scene 7) and the Cornell box (scene 6) with the current
# library, converted to gpurun_out/world_pmc_{7,6}.json (tools/world_pmc_json.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SCENE=7 bash tools/gpu_world_pmc.sh && python tools/world_pmc_json.py gpurun_out 7 > gpurun_out/world_pmc_7.json &&
SCENE=6 bash tools/gpu_world_pmc.sh && python tools/world_pmc_json.py gpurun_out 6 > gpurun_out/world_pmc_6.json
