# PC sampling (host trap, time-based) of one f64 trace launch: where the
# waves of the megakernel spend their time, per instruction.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCM:-host_trap} \
  --pc-sampling-unit ${PCU:-time} --pc-sampling-interval ${PCI:-1} \
  --output-format csv -d gpurun_out/pcs -o run -- python tools/prof_run.py f64 > gpurun_out/pcs.log 2>&1
ls -la gpurun_out/pcs >> gpurun_out/pcs.log 2>&1 || true
