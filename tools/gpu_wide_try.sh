# The per-lane walk on the 4-wide BVH (world_traversal=lane, the default for the globe) vs the
# binary BVH (lane2) vs the union walk: the world GPU tests (all three), then the globe, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_world.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/wide_world_tests.txt 2>&1; r=$?; tail -15 gpurun_out/wide_world_tests.txt; [ $r -eq 0 ] &&
for k in 1 2 3; do
  timeout -k 10 300 python tools/world_bench.py 7 world_traversal=lane world_traversal=lane2 2>&1 | grep -v amdgpu.ids \
    | sed -E 's/"W": .*"linear": false, //' | cut -c1-330 | sed "s/^/round $k /"
done
