# GPU check: smoke, GPU parity tests, bench, rocprofv3 kernel trace of bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 &&
timeout -k 10 300 python tools/phase_profile.py > gpurun_out/phase.log 2>&1
