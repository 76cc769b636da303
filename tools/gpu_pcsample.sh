# PC sampling (rocprofv3, beta) of one configs[1] render: per-instruction
# sample counts of the kernels (tools/pcs_summary.py).  WHICH = f64 (the
# megakernel) or wf64 (the wavefront engine); METHOD = host_trap | stochastic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
W=${WHICH:-f64}
M=${METHOD:-host_trap}
U=$([ "$M" = stochastic ] && echo cycles || echo time)
I=${INTERVAL:-$([ "$M" = stochastic ] && echo 1048576 || echo 100)}
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $M --pc-sampling-unit $U \
  --pc-sampling-interval $I --output-format csv -d gpurun_out/pcs_${W}_$M -o run \
  -- python tools/prof_run.py $W > gpurun_out/pcs_${W}_$M.log 2>&1
