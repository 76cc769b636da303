# BVH leaf size for the per-lane walk (RTW_MAX_LEAF_PRIMS builds: lib_l1 / lib (2) / lib_l3 / lib_l4):
# the world GPU tests through each build (bit identity vs the oracle fixtures), then the globe, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_world.txt
ENGINE=world SCENES=7 LIBS="lib lib_l1 lib_l3 lib_l4" TESTS="tests/test_gpu_world.py" ROUNDS=4 bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"W": 1200.*"linear": false, //' gpurun_out/ab_world.txt | cut -c1-330
