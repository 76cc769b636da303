# Leaf size 1 (lib_l1) vs 2 (lib): globe (per-lane walk) and scene 1 (union walk, 23 nodes), 6 alternations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_world.txt
ENGINE=world SCENES=7,1 LIBS="lib lib_l1" ROUNDS=6 bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"W": .*"linear": false, //' gpurun_out/ab_world.txt | cut -c1-200
