# Megakernel A/B of library builds (RTW_LIB_PATH): bench.py configs[1] lines
# (f64 headline + f32 variant), builds in LIBS alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
for r in 1 2 3; do
  for L in ${LIBS:-lib lib_b}; do
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-wavefront-variant \
      --no-world-variants --no-cpu-baseline > gpurun_out/mk_ab_cur.json 2>> gpurun_out/mk_ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/mk_ab_cur.json'));print('$L', d['value'], d['f32_hybrid_variant']['value'], d['roofline']['trace_ms_per_launch'])" >> gpurun_out/mk_ab.txt
  done
done
