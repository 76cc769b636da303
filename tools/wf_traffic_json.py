"""HBM traffic of one wavefront frame (wf_extend + wf_shade, every bounce
launch of the frame, + the drain wf_drain / wf_finish) from the FETCH_SIZE / WRITE_SIZE PMC passes of
tools/gpu_pmc_wf.sh -> profiles/<tag>/wf_traffic.json, read by bench.py for
wavefront_variant.roofline.traffic.  FETCH_SIZE is doubled (gfx950 tallies
128-B reads at 64 B, MI355X_MICROARCH.md §HBM); units are KB (rocprofv3).
Usage: python tools/wf_traffic_json.py FETCH_DIR WRITE_DIR OUT [frames]"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracinginoneweekend.zig_amd"))
import rtw_amd as R  # noqa: E402  (the library defaults the passes ran with: rtw_hip.h RTW_DEFAULT_WF_*)

fetch_dir, write_dir, out = sys.argv[1], sys.argv[2], sys.argv[3]
frames = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4].isdigit() else 1
KERNELS = ("wf_extend", "wf_shade", "wf_step", "wf_finish", "wf_drain")
FUSED = "--split" not in sys.argv  # the engine form the passes ran (params.wf_form)
SETS = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--sets=")), R.DEFAULT_WF_SETS)  # params.wf_sets
PASSES = next((int(a.split("=")[1]) for a in sys.argv if a.startswith("--passes=")), R.DEFAULT_WF_PASSES)  # params.wf_passes


def total(d, name):
    v, per = 0.0, {}
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
            if k and r["Counter_Name"] == name:
                x = float(r["Counter_Value"])
                v += x
                per[k] = per.get(k, 0.0) + x
    return v, per


fk, fper = total(fetch_dir, "FETCH_SIZE")
wk, wper = total(write_dir, "WRITE_SIZE")
if fk == 0 or wk == 0:
    sys.exit("no bounce-kernel counter rows")
res = {"config": {"width": 1200, "height": 675, "spp": 500, "precision": "f64", "engine": "wavefront",
                  "fused": FUSED, "sets": SETS, "wf_paths": 0,
                  "passes": PASSES if FUSED else 1, "bounces": 1},
       "fetch_size_kb_per_frame": fk / frames, "write_size_kb_per_frame": wk / frames,
       "per_kernel_bytes_per_frame": {k: (2 * fper.get(k, 0.0) + wper.get(k, 0.0)) * 1024 / frames for k in KERNELS},
       "traffic_bytes_per_frame": (2 * fk + wk) * 1024 / frames,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over one 1200x675x500 f64 "
                 "wavefront render (tools/prof_run.py wf64); bytes = 2*FETCH_SIZE + WRITE_SIZE (KB x 1024), "
                 "summed over every bounce launch of the frame (wf_step, or wf_extend + wf_shade) and its in-register "
                 "drain (wf_drain, or wf_finish with params.wf_drain RTW_WF_DRAIN_SLOTS)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
