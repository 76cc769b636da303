# Round-2 evidence: every GPU test, smoke(), the default bench line, rocprofv3
# kernel statistics of the bench command, PMC passes of the world kernel on
# the globe (scene 7) and Cornell (scene 6), and the megakernel's VALU passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02 -o run \
  -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 &&
SCENE=7 bash tools/gpu_world_pmc.sh && SCENE=6 bash tools/gpu_world_pmc.sh &&
TAG=r02v bash tools/gpu_pmc_valu.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_r02_fetch -o run \
  --pmc FETCH_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_r02_write -o run \
  --pmc WRITE_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_write.log 2>&1
