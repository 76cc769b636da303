# Round-2 evidence: GPU tests (incl. the full-frame configs[1] oracle check and
# configs[2] at 2000 spp), smoke(), the default bench line, the plain
# `python bench.py --gpus 2` launcher path (gloo, both ranks on the one GPU),
# and the rocprofv3 kernel statistics of the bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
TAG=${TAG:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
RTW_DIST_BACKEND=gloo RTW_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 \
  --no-world-variants > gpurun_out/dist_launch_gloo2.json 2> gpurun_out/dist_launch_gloo2.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run \
  -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
