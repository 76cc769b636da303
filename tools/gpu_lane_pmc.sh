# PMC passes of the globe (configs[4]) with the per-lane traversal beside the union walk.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
SCENE=7 OUT=7l CFG=world_traversal=lane bash tools/gpu_world_pmc.sh &&
python tools/world_pmc_json.py gpurun_out 7l > gpurun_out/world_pmc_7_lane.json &&
python -c "
import json
for f in ('profiles/r05/world_pmc_7.json', 'gpurun_out/world_pmc_7_lane.json'):
    d = json.load(open(f)); c = d['counters']
    print(f, d['dispatch_ms'], 'valu/wi', d['valu_per_wave_iteration'], 'salu/wi', d['salu_per_wave_iteration'],
          'busy', d['valu_busy_frac'], 'wait', d['wait_frac_of_wave_cycles'], 'vmem_rd', c.get('SQ_INSTS_VMEM_RD'),
          'lds', c.get('SQ_INSTS_LDS'), 'hbm', d['hbm_fetch_bytes'] + d['hbm_write_bytes'])
"
