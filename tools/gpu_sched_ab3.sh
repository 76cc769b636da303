# Globe (configs[4]) only: max-memory-clause scheduling (lib_s3) vs the default (lib), 6 alternations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_world.txt
ENGINE=world SCENES=7 LIBS="lib lib_s3" ROUNDS=6 bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"bvh.*"segments_per_sample"/"segments_per_sample"/' gpurun_out/ab_world.txt | cut -c1-140
