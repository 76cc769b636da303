import sys, json
sys.path.insert(0, 'tools')
from world_bench import run
for sc in (6, 1, 5, 3):
    for lin in (False, True):
        d = run(sc, linear=lin)
        print(d['name'], 'linear' if lin else 'bvh', d['ms'], 'ms', d['msamples_s'], 'Ms/s', flush=True)
