"""Launch timeline of the last wavefront frame in a rocprofv3 kernel trace,
per queue set: the kernels of each HIP stream / hardware queue, the frame
span, the time each set keeps the GPU busy, and the time in which kernels of
two (or more) sets run at once — the overlap the queue sets exist for
(DESIGN.md §6.2).
Usage: python tools/wf_overlap_summary.py <run_kernel_trace.csv> [json_out]"""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
              (r.get("Queue_Id"), r.get("Stream_Id"))) for r in rows if r.get("Kind", "KERNEL_DISPATCH") ==
             "KERNEL_DISPATCH"), key=lambda x: x[1])
short = lambda n: n.split("(")[0].split("<")[0].split("::")[-1].replace("void ", "")  # noqa: E731
# the last frame: from its queue sets' wf_generate launches (one per set:
# one per distinct queue / stream) to its last wf_check_drained
gens = [i for i, k in enumerate(ks) if short(k[0]) == "wf_generate"]
chk = [i for i, k in enumerate(ks) if short(k[0]) == "wf_check_drained"]
n_sets = len({ks[i][3] for i in gens})
seq = ks[gens[-n_sets]:chk[-1] + 1]
t0, t1 = seq[0][1], max(k[2] for k in seq)
span = (t1 - t0) / 1e6
sets = sorted({k[3] for k in seq if short(k[0]) == "wf_generate"})
sid = {q: i for i, q in enumerate(sets)}
busy = collections.defaultdict(float)
per = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
ev = []
for n, s, e, q in seq:
    i = sid.get(q, -1)
    per[i][short(n)][0] += 1
    per[i][short(n)][1] += (e - s) / 1e6
    ev += [(s, 1, i), (e, -1, i)]
ev.sort()
active = collections.Counter()
cover = [0.0] * (len(sets) + 2)  # time with exactly k sets running
last = t0
for t, d, i in ev:
    k = sum(1 for v in active.values() if v > 0)
    cover[min(k, len(cover) - 1)] += (t - last) / 1e6
    last = t
    active[i] += d
out = {"frame_span_ms": round(span, 3), "queue_sets": len(sets), "launches": len(seq),
       "ms_with_sets_running": {str(k): round(v, 3) for k, v in enumerate(cover) if v > 0},
       "overlap_ms": round(sum(cover[2:]), 3), "idle_ms": round(cover[0], 3),
       "per_set": {str(i): {k: {"launches": c, "busy_ms": round(t, 3)} for k, (c, t) in d.items()}
                   for i, d in sorted(per.items())}}
print(f"frame span {span:.3f} ms, {len(sets)} queue set(s) (queue/stream ids {sets}), {len(seq)} launches")
for k, v in enumerate(cover):
    if v > 0:
        print(f"  {v:9.3f} ms with {k} set(s) running")
for i, d in sorted(per.items()):
    print(f"  set {i}: " + ", ".join(f"{k} {c} x = {t:.3f} ms" for k, (c, t) in sorted(d.items(), key=lambda x: -x[1][1])))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
