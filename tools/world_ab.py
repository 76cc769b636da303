"""In-process A/B of world-kernel knobs on the GPU box:
python tools/world_ab.py SCENES 'ENV=a,ENV2=b;ENV=c' [rounds]
Each configuration (a ';'-separated list of comma-separated env settings) is
timed with tools/world_bench.run (best of 3 HIP-event timed renders), the
configurations interleaved over `rounds` rounds; prints one JSON line per run."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from world_bench import run  # noqa: E402

scenes = [int(x) for x in sys.argv[1].split(",")]
confs = [dict(kv.split("=", 1) for kv in c.split(",") if kv) for c in sys.argv[2].split(";")]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
keys = sorted({k for c in confs for k in c})
for r in range(rounds):
    for sc in scenes:
        for c in confs:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(c)
            o = run(sc)
            print(json.dumps({"round": r, "conf": c, "scene": sc, "ms": o["ms"], "msamples_s": o["msamples_s"],
                              "visits": o["node_visits_per_segment"], "tests": o["prim_tests_per_segment"]}),
                  flush=True)
