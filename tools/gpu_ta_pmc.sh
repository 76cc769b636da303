# Is the per-lane BVH walk bound by the vector memory pipeline (TA address processing of
# divergent per-lane loads)?  One PMC pass per traversal over one globe render
# (tools/world_prof_run.py 7): TA / TD busy, TA stalls by the cache, TCP accesses and stalls.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for T in lane lane2 union; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ta_$T -o run \
    --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum \
      TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum \
    -- python tools/world_prof_run.py 7 1 world_traversal=$T > gpurun_out/ta_$T.log 2>&1 || exit 1
done
ls gpurun_out/ta_lane
