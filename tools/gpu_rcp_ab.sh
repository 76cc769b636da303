# (A/B of a change that was not adopted: the rcp_rn source it measured is in profiles/r02/rcp_ab.txt only)
# rcp_rn (RTW_FAST_RCP=1, lib) vs the IEEE reciprocal (lib_o): every GPU test
# on lib (incl. the device bit check of rcp_rn), then the megakernel and the
# world kernel A/B, builds alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_rcp.log 2>&1 &&
LIBS="lib_o lib" bash tools/gpu_mk_lib_ab.sh &&
LIBS="lib_o lib" SCENES=7,6 bash tools/gpu_world_lib_ab.sh
