# PMC evidence for the default f64 trace kernel (configs[1]): the VALU-issue
# passes (tools/gpu_pmc_valu.sh) and the HBM traffic passes (FETCH_SIZE and
# WRITE_SIZE in separate runs, MI355X_MICROARCH.md HBM section).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01v} bash tools/gpu_pmc_valu.sh &&
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run \
  --pmc FETCH_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run \
  --pmc WRITE_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_write.log 2>&1
