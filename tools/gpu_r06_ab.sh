#!/bin/bash
# Round 6: every GPU test through this tree's build, then A/Bs of round 5's
# library (lib_r5, built from the round-5 sources) against this tree's (lib),
# alternated ROUNDS times in separate processes: the megakernel (bench.py
# configs[1] f64 + f32 lines), the wavefront engine (tools/wf_bench.py) and the
# world kernel (tools/world_bench.py: globe, Cornell, scene 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
LIBS=${LIBS:-lib_r5 lib}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
    > gpurun_out/r06_tests.txt 2>&1 || { tail -40 gpurun_out/r06_tests.txt; exit 1; }
  tail -2 gpurun_out/r06_tests.txt
fi
OUT=gpurun_out/r06_ab.txt
: > $OUT
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in $LIBS; do
    E="RTW_LIB_PATH=$P/$L/librtw_hip.so"
    if [[ "${ENGINES:-mk wf world}" == *mk* ]]; then
      env $E timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-wavefront-variant --no-world-variants \
        --no-cpu-baseline > gpurun_out/ab_cur.json 2>> gpurun_out/r06_ab.err || exit 1
      python -c "import json;d=json.load(open('gpurun_out/ab_cur.json'));print('mk $L $r', d['value'], \
d['f32_hybrid_variant']['value'], d['roofline']['trace_ms_per_launch'])" >> $OUT
    fi
    if [[ "${ENGINES:-mk wf world}" == *wf* ]]; then
      env $E timeout -k 10 300 python tools/wf_bench.py 3 2>> gpurun_out/r06_ab.err | sed "s/^/wf $L $r /" >> $OUT || exit 1
    fi
    if [[ "${ENGINES:-mk wf world}" == *world* ]]; then
      env $E WORLD_REPS=5 timeout -k 10 300 python tools/world_bench.py ${SCENES:-7,6,1} 2>> gpurun_out/r06_ab.err \
        | sed "s/^/world $L $r /" >> $OUT || exit 1
    fi
    echo "round $r $L done"
  done
done
python tools/ab_summary.py $OUT
