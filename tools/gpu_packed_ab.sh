# Per-lane walk with the child refs packed into the lower bounds' low bits (three 16-B node loads
# instead of four): the globe with lib_m (packed) vs lib_m2 (the same -DRTW_MEASURE library,
# RTW_WORLD_UNPACKED=1), alternated processes, best of WORLD_REPS renders each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_world.txt
ENGINE=world SCENES=7 LIBS="lib_m lib_m2" ENVS="lib_m2:RTW_WORLD_UNPACKED=1" ROUNDS=${ROUNDS:-4} WORLD_REPS=${WORLD_REPS:-12} \
  bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"W": .*"linear": false, //' gpurun_out/ab_world.txt | cut -c1-200
