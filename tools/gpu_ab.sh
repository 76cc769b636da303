# A/B of library builds (RTW_LIB_PATH) on the GPU box, alternated in separate
# processes, optionally after GPU tests through each candidate build.
# Replaces round 2's per-experiment launchers (gpu_mk_lib_ab.sh,
# gpu_world_lib_ab.sh, gpu_wf_lib_ab.sh, gpu_world_*.sh, gpu_wf_*_ab.sh, ...:
# `git show 9194c38:tools/<name>` has them).
#   ENGINE=mk     bench.py configs[1] lines (f64 headline + f32 variant)
#   ENGINE=wf     tools/wf_bench.py (configs[3], the wavefront engine)
#   ENGINE=world  tools/world_bench.py (SCENES, default "7,6": globe, Cornell)
#   LIBS="lib lib_x"  build directories under raytracinginoneweekend.zig_amd
#                 (make BUILD=build_x LIBDIR=lib_x EXTRA=-D... lib_x/librtw_hip.so)
#   TESTS="tests/test_gpu_parity.py ..."  pytest -m gpu selection run through
#                 every build of LIBS before the timing (bit identity)
#   ROUNDS=3      alternations;  ENVS="lib:RTW_X=1"  extra env per build
#   PMC="lib_x"   afterwards, the VALU-issue PMC passes of configs[1]
#                 (tools/gpu_pmc_valu.sh) through each of these builds, TAG=ab_<build>
# Output: gpurun_out/ab_<ENGINE>.txt (one line per build and round).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
ENGINE=${ENGINE:-mk}
OUT=gpurun_out/ab_${ENGINE}.txt
envs_of() {  # extra environment of build $1 from ENVS ("lib:K=V,K2=V2 lib_x:K=V")
  for e in ${ENVS:-}; do
    [ "${e%%:*}" = "$1" ] && echo "${e#*:}" | tr ',' ' '
  done
}
if [ -n "${TESTS:-}" ]; then
  for L in ${LIBS:-lib}; do
    env $(envs_of $L) RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 \
      --timeout-method thread -m gpu $TESTS > gpurun_out/ab_tests_$L.txt 2>&1 || exit 1
    tail -1 gpurun_out/ab_tests_$L.txt | sed "s/^/tests $L: /" >> $OUT
  done
fi
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in ${LIBS:-lib lib_b}; do
    E="$(envs_of $L) RTW_LIB_PATH=$P/$L/librtw_hip.so"
    case $ENGINE in
      mk)
        env $E timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-wavefront-variant --no-world-variants \
          --no-cpu-baseline > gpurun_out/ab_cur.json 2>> gpurun_out/ab.err || exit 1
        python -c "import json;d=json.load(open('gpurun_out/ab_cur.json'));print('$L round $r', d['value'], \
d['f32_hybrid_variant']['value'], d['roofline']['trace_ms_per_launch'])" >> $OUT ;;
      wf)
        env $E timeout -k 10 300 python tools/wf_bench.py 2>> gpurun_out/ab.err | sed "s/^/$L round $r /" >> $OUT || exit 1 ;;
      world)
        env $E timeout -k 10 300 python tools/world_bench.py ${SCENES:-7,6} 2>> gpurun_out/ab.err \
          | sed "s/^/$L round $r /" >> $OUT || exit 1 ;;
    esac
  done
done
for L in ${PMC:-}; do
  RTW_LIB_PATH=$P/$L/librtw_hip.so TAG=ab_$L bash tools/gpu_pmc_valu.sh || exit 1
done
cat $OUT
