# Packed refs: one payload byte per lower bound gathered by two v_perm_b32 (lib) vs 6 bits per bound
# gathered by ands / shifts (lib_p6, the previous commit): world GPU tests through lib, then the globe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/packed8_world_tests.txt 2>&1; r=$?; tail -2 gpurun_out/packed8_world_tests.txt; [ $r -eq 0 ] &&
rm -f gpurun_out/ab_world.txt &&
ENGINE=world SCENES=7 LIBS="lib lib_p6" ROUNDS=5 WORLD_REPS=12 bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"W": .*"linear": false, //' gpurun_out/ab_world.txt | cut -c1-120
