#!/bin/bash
# Round 6: the wavefront frame's PMC traffic against its queue configuration
# (is the 0.77x of the algorithmic bytes the smaller queue footprint's L2 reuse?):
# FETCH_SIZE / WRITE_SIZE passes of tools/prof_run.py wf64 at the round-5 defaults
# (786,432 paths, 8 passes) and at 655,360 paths with 8 passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "786432 8" "655360 8"; do
  set -- $cfg
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wfl2_${1}_${2}_$c -o run \
      --pmc $c -- python tools/prof_run.py wf64 1 wf_paths=$1 wf_passes=$2 > gpurun_out/wfl2_${1}_${2}_$c.log 2>&1 || exit 1
  done
  python tools/wf_traffic_json.py gpurun_out/wfl2_${1}_${2}_FETCH_SIZE gpurun_out/wfl2_${1}_${2}_WRITE_SIZE \
    gpurun_out/wfl2_${1}_${2}.json --passes=$2 | python -c "import json,sys; d=json.load(sys.stdin); print('paths $1 passes $2', d['traffic_bytes_per_frame'], d['per_kernel_bytes_per_frame'])"
done
