# The world kernel's translation unit with LLVM's max-memory-clause scheduler (lib_s3) vs the
# default (lib), after the round's per-lane walk changes: globe + Cornell, best of 12, 6 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_world.txt
ENGINE=world SCENES=7,6 LIBS="lib lib_s3" ROUNDS=6 WORLD_REPS=12 bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"W": .*"linear": false, //' gpurun_out/ab_world.txt | cut -c1-120
