# Round evidence on the GPU box, in stages (STAGES, default "tests pmc bench"):
#   tests  every GPU test (pytest -m gpu) + smoke()            -> gpurun_out/pytest_gpu.log, smoke.log
#   pmc    the PMC passes the bench line reads: megakernel VALU issue
#          (gpu_pmc_valu.sh) and HBM traffic (FETCH_SIZE, WRITE_SIZE in separate
#          passes), wavefront traffic (gpu_pmc_wf.sh), world kernel on the globe
#          and Cornell (gpu_world_pmc.sh)
#   bench  the default bench line + rocprofv3 --kernel-trace --stats of the same command
# TAG names the rocprofv3 output directories (default r03).  Every GPU step has
# its own time limit and the chain stops at the first failure.
# Replaces round 2's gpu_r02_*.sh / gpu_bench_profile.sh / gpu_round.sh
# (`git show 9194c38:tools/<name>`).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
TAG=${TAG:-r03}
for stage in ${STAGES:-tests pmc bench}; do
  case $stage in
    tests)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v -s --durations=15 --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 &&
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1 ;;
    pmc)
      TAG=${TAG}v bash tools/gpu_pmc_valu.sh &&
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_fetch -o run \
        --pmc FETCH_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_fetch.log 2>&1 &&
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_write -o run \
        --pmc WRITE_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_write.log 2>&1 &&
      bash tools/gpu_pmc_wf.sh &&
      SCENE=7 bash tools/gpu_world_pmc.sh && SCENE=6 bash tools/gpu_world_pmc.sh || exit 1 ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run \
        -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit 1 ;;
  esac
done
