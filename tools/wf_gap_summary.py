"""Launch-level timeline of the last wavefront frame in a rocprofv3 kernel
trace (fused or split engine): frame span, busy time per kernel name, and the
idle time between consecutive kernels (dispatch gaps).
Usage: python tools/wf_gap_summary.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows),
            key=lambda x: x[1])
gens = [i for i, k in enumerate(ks) if "wf_generate" in k[0]]
seq = ks[gens[-1]:]
fin = [i for i, k in enumerate(seq) if "wf_finish" in k[0] or "wf_check_drained" in k[0]]
seq = seq[: fin[-1] + 1] if fin else seq
span = (seq[-1][2] - seq[0][1]) / 1e6
busy = collections.defaultdict(lambda: [0, 0.0])
for n, s, e in seq:
    short = n.split("(")[0].split("<")[0].split("::")[-1]
    busy[short][0] += 1
    busy[short][1] += (e - s) / 1e6
gaps = [(b[1] - a[2]) / 1e3 for a, b in zip(seq, seq[1:])]
print(f"frame span {span:.3f} ms, {len(seq)} launches, busy {sum(v[1] for v in busy.values()):.3f} ms, "
      f"idle between launches {sum(g for g in gaps if g > 0) / 1e3:.3f} ms "
      f"(mean gap {sum(gaps) / len(gaps):.2f} us, max {max(gaps):.1f} us)")
for k, (c, t) in sorted(busy.items(), key=lambda x: -x[1][1]):
    print(f"  {k:24s} {c:6d} launches {t:9.3f} ms  mean {1e3 * t / c:8.2f} us")
