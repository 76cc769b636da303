set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=20
mkdir -p gpurun_out
for g in 1 2 4 16; do
  echo "grid x$g" >> gpurun_out/wf_grid.log
  RTW_WF_GRID=$g timeout -k 10 200 python tools/wf_sweep.py f64,f32 524288,1048576,2097152 >> gpurun_out/wf_grid.log 2>&1 || exit 1
done
