# Final round-2 evidence, pass 1: every GPU test, smoke(), and the PMC passes
# the bench line reads (megakernel VALU + traffic, wavefront traffic).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
TAG=r02v bash tools/gpu_pmc_valu.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_r02_fetch -o run \
  --pmc FETCH_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_r02_write -o run \
  --pmc WRITE_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_write.log 2>&1 &&
bash tools/gpu_pmc_wf.sh
