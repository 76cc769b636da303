"""One render of one world scene (for rocprofv3 PMC passes):
python tools/world_prof_run.py SCENE [reps] [cfg]  (scene settings of main.zig; cfg: comma-separated
rtw_params fields as tools/world_bench.py, e.g. world_traversal=lane)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from world_bench import run  # noqa: E402

if __name__ == "__main__":
    sc = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    kw = {}
    for kv in (sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[3] != "-" else []):
        k, v = kv.split("=")
        kw[k] = int(v) if v.isdigit() else v
    print(run(sc, reps=int(sys.argv[2]) if len(sys.argv) > 2 else 1, **kw), flush=True)
