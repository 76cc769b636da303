# Bench line + its rocprofv3 kernel statistics (after the PMC evidence files
# under profiles/r02 are in place: the line reads them).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02c -o run \
  -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
