# Wavefront engine: queue-capacity sweep + rocprofv3 kernel stats of one config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-wf1}
RTW_WF_TIMEOUT_S=20 timeout -k 10 300 python tools/wf_sweep.py f64,f32 262144,524288,1048576,2097152,4194304 > gpurun_out/wf_sweep_$TAG.log 2>&1 &&
REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python tools/wf_sweep.py f64 1048576 > gpurun_out/wf_prof_$TAG.log 2>&1
