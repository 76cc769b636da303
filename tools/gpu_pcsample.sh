# PC sampling of one configs[1] f64 megakernel render (rocprofv3 beta):
# per-instruction sample counts of trace_kernel, for attributing issue time to
# source lines (tools/pcs_lines.py).  METHOD=stochastic|host_trap.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
M=${METHOD:-host_trap}
U=$([ "$M" = stochastic ] && echo cycles || echo time)
I=${INTERVAL:-$([ "$M" = stochastic ] && echo 1048576 || echo 50)}
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
  --pc-sampling-interval $I --output-format csv -d gpurun_out/pcs_$M -o run \
  -- python tools/prof_run.py f64 > gpurun_out/pcs_$M.log 2>&1
