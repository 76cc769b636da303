# Round-2 evidence, second pass: wavefront PMC traffic (wf_extend retuned),
# then the bench line (world rooflines from profiles/r02) and its rocprofv3
# kernel statistics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
bash tools/gpu_pmc_wf.sh &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02b -o run \
  -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
