"""Per-phase summary of a wavefront frame from a rocprofv3 kernel trace:
mean extend / shade durations by iteration range (last frame in the trace)."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows),
            key=lambda x: x[1])
gens = [i for i, k in enumerate(ks) if "wf_generate" in k[0]]
seq = ks[gens[-1]:]
ext = [k for k in seq if "wf_extend" in k[0]]
shd = [k for k in seq if "wf_shade" in k[0]]
print(f"iterations {len(ext)}  frame span {(seq[-1][2] - seq[0][1]) / 1e6:.2f} ms  "
      f"extend total {sum(k[2] - k[1] for k in ext) / 1e6:.2f} ms  shade total {sum(k[2] - k[1] for k in shd) / 1e6:.2f} ms")
n = len(ext)
edges = sorted(set([0, 50, n // 4, n // 2, (3 * n) // 5, (7 * n) // 10, (4 * n) // 5, (9 * n) // 10, n]))
for lo, hi in zip(edges, edges[1:]):
    if hi <= lo:
        continue
    e = statistics.mean((k[2] - k[1]) / 1e3 for k in ext[lo:hi])
    s = statistics.mean((k[2] - k[1]) / 1e3 for k in shd[lo:hi])
    g = statistics.mean((shd[i][1] - ext[i][2]) / 1e3 for i in range(lo, min(hi, len(shd))))
    print(f"  iters {lo:5d}-{hi:5d}: extend {e:7.1f} us  shade {s:7.1f} us  gap {g:5.1f} us")
