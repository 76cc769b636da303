"""Per-kernel totals of rocprofv3 --pmc passes over one wavefront render: for
each kernel name (wf_step, wf_drain, wf_finish, ...) the counter sums over
its dispatches and per-dispatch means of the wave / issue ratios.
Usage: python tools/wf_kernel_pmc.py <pass_dir> [<pass_dir> ...]"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((d, r.get("Dispatch_Id", "")))
for k, c in sorted(agg.items()):
    print(f"{k}: {len(disp[k])} dispatch-passes")
    for n, v in sorted(c.items()):
        print(f"  {n:24s} {v:.4g}")
    if c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
        print(f"  VALU per wave {c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}, SALU per wave {c.get('SQ_INSTS_SALU', 0) / c['SQ_WAVES']:.0f}")
    if c.get("SQ_WAVE_CYCLES"):
        print(f"  wait share {c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES']:.3f}, "
              f"active-inst share {c.get('SQ_ACTIVE_INST_ANY', 0) / c['SQ_WAVE_CYCLES']:.3f}")
