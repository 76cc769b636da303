# Wavefront queue-capacity sweep with the in-register drain (RTW_WF_FINISH=1)
# and two drain thresholds at the default capacity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
timeout -k 10 400 python tools/wf_sweep.py f64,f32 524288,1048576,2097152,4194304 > gpurun_out/wf_sweep2.txt 2>&1 &&
RTW_WF_FINISH=0.5 timeout -k 10 200 python tools/wf_sweep.py f64 1048576 | sed 's/^/finish<0.5n /' >> gpurun_out/wf_sweep2.txt 2>&1 &&
RTW_WF_FINISH=0.9 timeout -k 10 200 python tools/wf_sweep.py f64 1048576 | sed 's/^/finish<0.9n /' >> gpurun_out/wf_sweep2.txt 2>&1
