"""Summary of tools/gpu_r06_ab.sh's A/B record: per engine, configuration and
build, the timings of every round and their mean (ms; lower is faster).
Usage: python tools/ab_summary.py gpurun_out/r06_ab.txt"""
import collections
import json
import sys

acc = collections.defaultdict(list)
for line in open(sys.argv[1]):
    parts = line.split(" ", 3)
    if len(parts) < 4:
        continue
    eng, lib, rnd, rest = parts
    if eng == "mk":
        v64, v32, ms = rest.split()
        acc[("mk f64 Msamples/s", lib)].append(float(v64))
        acc[("mk f32 Msamples/s", lib)].append(float(v32))
        acc[("mk trace ms", lib)].append(float(ms))
    elif eng == "wf":  # "wavefront f64 [cfg] 49.2 ms 8228 Msamples/s"
        w = rest.split()
        i = w.index("ms")
        cfg = " ".join(w[2:i - 1]) or "-"
        acc[("wf ms " + cfg, lib)].append(float(w[i - 1]))
    elif eng == "world":
        d = json.loads(rest)
        acc[(f"world scene {d['scene']} ms", lib)].append(float(d["ms"]))
for (k, lib), v in sorted(acc.items()):
    print(f"{k:28s} {lib:8s} {' '.join(f'{x:9.2f}' for x in v)}   mean {sum(v) / len(v):9.2f}")
