"""One render of one world scene (for rocprofv3 PMC passes):
python tools/world_prof_run.py SCENE [reps]  (scene settings of main.zig)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from world_bench import run  # noqa: E402

if __name__ == "__main__":
    sc = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    print(run(sc, reps=int(sys.argv[2]) if len(sys.argv) > 2 else 1), flush=True)
