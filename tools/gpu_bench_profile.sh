# Round-end evidence: GPU tests, the default bench line, the rocprofv3 kernel
# summary of the same bench command, and the HBM-traffic PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md §HBM).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run \
  -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_fetch -o run \
  --pmc FETCH_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_write -o run \
  --pmc WRITE_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_write.log 2>&1
