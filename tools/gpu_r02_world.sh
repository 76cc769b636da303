# World kernel evidence: timings of scenes 7 (configs[4] globe) and 6
# (Cornell) + the PMC passes of the globe render.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/world_bench.py 7,6 > gpurun_out/world_bench.txt 2> gpurun_out/world_bench.err &&
SCENE=7 bash tools/gpu_world_pmc.sh
