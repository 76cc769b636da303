"""Per-launch HBM traffic of the f64 trace kernel from the FETCH_SIZE / WRITE_SIZE
PMC passes (tools/gpu_evidence.sh, stage pmc) -> profiles/<tag>/traffic.json, read by
bench.py for roofline.traffic.  FETCH_SIZE is doubled (gfx950 tallies 128-B
reads at 64 B, MI355X_MICROARCH.md §HBM); units are KB (rocprofv3)."""
import csv
import glob
import json
import sys

fetch_dir, write_dir, out = sys.argv[1], sys.argv[2], sys.argv[3]


def total(d, name):
    v, n = 0.0, set()
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" in r["Kernel_Name"] and r["Counter_Name"] == name:
                v += float(r["Counter_Value"])
                n.add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    return v, max(1, len(n))


fk, nf = total(fetch_dir, "FETCH_SIZE")
wk, nw = total(write_dir, "WRITE_SIZE")
res = {"config": {"width": 1200, "height": 675, "spp": 500, "precision": "f64"},
       "fetch_size_kb_per_launch": fk / nf, "write_size_kb_per_launch": wk / nw,
       "traffic_bytes_per_launch": (2 * fk / nf + wk / nw) * 1024,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over one 1200x675x500 f64 "
                 "render (tools/prof_run.py); bytes = 2*FETCH_SIZE + WRITE_SIZE (KB x 1024)"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
