# HBM traffic of the wavefront engine's bounce kernels (BASELINE configs[3]):
# FETCH_SIZE and WRITE_SIZE in separate PMC passes over one f64 frame.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_fetch -o run \
  --pmc FETCH_SIZE -- python tools/prof_run.py wf64 > gpurun_out/wf_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wf_write -o run \
  --pmc WRITE_SIZE -- python tools/prof_run.py wf64 > gpurun_out/wf_write.log 2>&1 &&
python tools/wf_traffic_json.py gpurun_out/wf_fetch gpurun_out/wf_write gpurun_out/wf_traffic.json
