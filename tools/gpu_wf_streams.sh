# the wavefront's queue sets overlap with many other streams in the process: kernel traces
# of the configs[1] wavefront frame with 0 and 12 extra torch streams bound before the library's side
# stream, summarised per queue set (tools/wf_overlap_summary.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out/ev
for n in 0 12; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wfs_$n -o run \
    -- python tools/wf_streams_run.py $n > gpurun_out/wfs_$n.log 2>&1 || exit 1
  grep "extra streams" gpurun_out/wfs_$n.log
  python tools/wf_overlap_summary.py gpurun_out/wfs_$n/run_kernel_trace.csv gpurun_out/ev/wf_overlap_streams$n.json | tail -8 || exit 1
done
