# Refresh of the diagnostic profiles for the current kernels: world register
# budgets, world BVH vs linear, trace-kernel phase stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/world_ab.log
bash tools/gpu_world_ab.sh &&
timeout -k 10 300 python tools/world_linear_ab.py > gpurun_out/world_linear_ab.log 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1
