#!/bin/bash
# Round 6: the world GPU tests through the current build, then an A/B of the
# world kernel (globe, Cornell, scene 1) between builds (LIBS, default
# "lib_r5 lib": round 5's library vs this tree's), alternated ROUNDS times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_world.py \
    > gpurun_out/r06_world_tests.txt 2>&1 || { tail -30 gpurun_out/r06_world_tests.txt; exit 1; }
  tail -3 gpurun_out/r06_world_tests.txt
fi
OUT=gpurun_out/r06_world_ab.txt
: > $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in ${LIBS:-lib_r5 lib}; do
    RTW_LIB_PATH=$P/$L/librtw_hip.so WORLD_REPS=5 timeout -k 10 300 python tools/world_bench.py ${SCENES:-7,6,1} \
      2>> gpurun_out/r06_world_ab.err | sed "s/^/$L round $r /" >> $OUT || exit 1
  done
done
python - <<'PY'
import json, collections
acc = collections.defaultdict(list)
for l in open("gpurun_out/r06_world_ab.txt"):
    lib, _, rnd, js = l.split(" ", 3)
    d = json.loads(js)
    acc[(d["scene"], lib)].append(d["ms"])
for (sc, lib), v in sorted(acc.items()):
    print(f"scene {sc} {lib:8s} ms {' '.join(f'{x:.2f}' for x in v)}  mean {sum(v)/len(v):.2f}")
PY
