"""Summarise the world-kernel PMC passes (tools/gpu_world_pmc.sh) of one
render: counters summed over the world_kernel dispatch(es) of the timed
render (the last dispatch of each pass), plus derived issue/wait fractions
and HBM bytes (FETCH_SIZE doubled per the gfx950 rule of
MI355X_MICROARCH.md, WRITE_SIZE as read; both in KB).
python tools/world_pmc_json.py gpurun_out SCENE > profiles/r02/world_pmc_globe.json"""
import collections
import csv
import glob
import json
import sys

root, scene = sys.argv[1], sys.argv[2]
c = {}
disp = {}
for tag in "abcfw":
    for f in glob.glob(f"{root}/wpmc_{scene}_{tag}/*counter_collection.csv"):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "world_kernel<0" not in r["Kernel_Name"]:
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        last = max(per)
        c.update(per[last])
        disp[tag] = last
simds, clk_ghz = 1024, 2.4
wave_cyc = c["SQ_WAVE_CYCLES"]
out = {"scene": int(scene), "counters": {k: c[k] for k in sorted(c)},
       "valu_busy_frac": c["SQ_ACTIVE_INST_VALU"] * 4 / (simds * c["GRBM_GUI_ACTIVE"]) if "GRBM_GUI_ACTIVE" in c else None,
       "wait_frac_of_wave_cycles": c["SQ_WAIT_ANY"] / wave_cyc,
       "issue_frac_of_wave_cycles": c["SQ_ACTIVE_INST_ANY"] / wave_cyc,
       "hbm_fetch_bytes": c.get("FETCH_SIZE", 0) * 1024 * 2, "hbm_write_bytes": c.get("WRITE_SIZE", 0) * 1024,
       "note": "valu_busy_frac = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE); FETCH_SIZE doubled "
               "(gfx950), FETCH/WRITE_SIZE in KB"}
print(json.dumps(out, indent=1))
