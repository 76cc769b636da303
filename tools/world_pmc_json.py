"""Summarise the world-kernel PMC passes (tools/gpu_world_pmc.sh) of one
render: counters of the timed render's world_kernel dispatch (the last one
of each pass), the dispatch time and clock, the VALU-issue figures and the
HBM bytes (FETCH_SIZE doubled per the gfx950 rule of MI355X_MICROARCH.md,
WRITE_SIZE as read; both counters are in KB).  bench.py reads the result
for world_variant roofline (profiles/r02/world_pmc_<scene>.json).
python tools/world_pmc_json.py gpurun_out SCENE > profiles/r02/world_pmc_SCENE.json"""
import collections
import csv
import glob
import json
import sys

SIMDS = 256 * 4
root, scene = sys.argv[1], sys.argv[2]
c, ms, tpass = {}, None, {}
for tag in "abcfwt":
    d = f"{root}/wpmc_{scene}_{tag}"
    if tag == "t" and not glob.glob(f"{d}/*counter_collection.csv"):
        continue  # (older runs: no TA / TD pass)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "world_kernel<0" in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
                names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    last = max(per)
    if tag == "t":  # its own GRBM_GUI_ACTIVE: the busy shares are over this pass's dispatch
        tpass = dict(per[last])
        continue
    c.update(per[last])
    if tag == "b":
        for f in glob.glob(f"{d}/*kernel_trace.csv"):
            for r in csv.DictReader(open(f)):
                if int(r["Dispatch_Id"]) == last:
                    ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        kernel = names[last]
run = None
for line in open(f"{root}/wpmc_{scene}_b.log"):
    if line.startswith("{"):
        run = json.loads(line.replace("'", '"').replace("False", "false").replace("True", "true"))
segments = run["segments_per_sample"] * run["W"] * run["H"] * run["spp"]
cyc = c["GRBM_GUI_ACTIVE"] / 8  # per-XCD counter summed over the 8 XCDs
clock = cyc / (ms * 1e-3)
out = {"what": f"PMC passes of ONE world_kernel dispatch (scene {run['scene']}, {run['name']}, {run['W']}x{run['H']}x"
               f"{run['spp']}), rocprofv3 --pmc, one pass per counter set (tools/gpu_world_pmc.sh)",
       "scene": run["scene"], "config": {k: run[k] for k in ("world_traversal", "world_waves") if k in run},
       "kernel": kernel, "dispatch_ms": ms, "clock_ghz": round(clock / 1e9, 3),
       "segments": round(segments), "counters": {k: c[k] for k in sorted(c)},
       "valu_per_wave_iteration": round(c["SQ_INSTS_VALU"] / (segments / 64)),
       "salu_per_wave_iteration": round(c["SQ_INSTS_SALU"] / (segments / 64)),
       "valu_busy_frac": round(c["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc), 4),
       "wait_frac_of_wave_cycles": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
       "hbm_fetch_bytes": c["FETCH_SIZE"] * 1024 * 2, "hbm_write_bytes": c["WRITE_SIZE"] * 1024,
       # vector memory pipeline: TA (address processing, average over instances) and TD (data
       # return, summed over the 256 CUs' instances) busy cycles over the dispatch's cycles
       **({"ta_busy_frac": round(tpass["TA_BUSY_avr"] / (tpass["GRBM_GUI_ACTIVE"] / 8), 4),
           "td_busy_frac": round(tpass["TD_TD_BUSY_sum"] / 256 / (tpass["GRBM_GUI_ACTIVE"] / 8), 4),
           "vmem_counters": {k: tpass[k] for k in sorted(tpass)}} if tpass else {}),
       "note": "valu_busy_frac = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8); a wave64 VALU "
               "instruction occupies its SIMD for ~4 cycles, so the issue roof is 1024 x clock / 4 wave-instructions/s"}
print(json.dumps(out, indent=1))
