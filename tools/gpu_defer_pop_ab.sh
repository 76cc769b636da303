# Per-lane walk stack pops that do not wait on their LDS read in the popping step (lib) vs the
# previous commit (lib_pv): world GPU tests through lib, then the globe, best of 12, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/defer_world_tests.txt 2>&1; r=$?; tail -2 gpurun_out/defer_world_tests.txt; [ $r -eq 0 ] &&
rm -f gpurun_out/ab_world.txt &&
ENGINE=world SCENES=7 LIBS="lib lib_pv" ROUNDS=5 WORLD_REPS=12 bash tools/gpu_ab.sh > /dev/null &&
sed -E 's/"W": .*"linear": false, //' gpurun_out/ab_world.txt | cut -c1-120
