# PMC passes over one config-2 render per precision (separate from any trace run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_${TAG}_a -o run \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -- python tools/prof_run.py both > gpurun_out/pmc_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_${TAG}_b -o run \
  --pmc FETCH_SIZE \
  -- python tools/prof_run.py both > gpurun_out/pmc_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_${TAG}_c -o run \
  --pmc WRITE_SIZE \
  -- python tools/prof_run.py both > gpurun_out/pmc_c.log 2>&1
