# Megakernel A/B of (library build, env) configurations: CONFS entries are
# LIB or LIB+ENV=VALUE (e.g. lib_k+RTW_CLUSTER_FILL=1), alternated in
# separate processes; bench.py configs[1] f64 / f32 lines; optional counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
for r in 1 2 3; do
  for C in ${CONFS:-lib lib_k}; do
    L=${C%%+*}; E=""; [ "$C" != "$L" ] && E=${C#*+}
    env $E RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-wavefront-variant \
      --no-world-variants --no-cpu-baseline > gpurun_out/mk_ab_cur.json 2>> gpurun_out/mk_ab.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/mk_ab_cur.json'));print('$C', d['value'], d['f32_hybrid_variant']['value'], d['roofline']['trace_ms_per_launch'])" >> gpurun_out/mk_ab.txt
  done
done
