# Final round-2 evidence, pass 1b: every GPU test, smoke(), and all PMC passes
# the bench line reads (megakernel VALU + traffic, wavefront traffic, world
# kernel on the globe and Cornell).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
bash tools/gpu_r02_final_a.sh &&
SCENE=7 bash tools/gpu_world_pmc.sh && SCENE=6 bash tools/gpu_world_pmc.sh
