# Per-lane walk yield threshold after the round's walk changes: 16 (default, lib_m) vs 8 / 12 / 24
# (copies of the -DRTW_MEASURE library with RTW_WORLD_YIELD), globe, best of 12, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_world.txt
ENGINE=world SCENES=7 LIBS="lib_m lib_y8 lib_y12 lib_y24" ENVS="lib_y8:RTW_WORLD_YIELD=8 lib_y12:RTW_WORLD_YIELD=12 lib_y24:RTW_WORLD_YIELD=24" \
  ROUNDS=4 WORLD_REPS=12 bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"W": .*"linear": false, //' gpurun_out/ab_world.txt | cut -c1-120
