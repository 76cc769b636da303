"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel dispatch, counter totals."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if "trace_kernel" not in r["Kernel_Name"]:
                continue
            k = ("f32" if "float" in r["Kernel_Name"] else "f64", r["Counter_Name"])
            agg[k] += float(r["Counter_Value"])
        for k, v in sorted(agg.items()):
            print(d.split("/")[-1], k[0], k[1], f"{v:.4g}")
