# The per-lane walk's register budget after the round's walk changes: 4 waves/SIMD (default, 80-B spill)
# vs 3 (no spill): globe, best of 12, in-process alternation of the two params.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for k in 1 2 3 4; do
  WORLD_REPS=12 timeout -k 10 300 python tools/world_bench.py 7 - world_waves=3 2>&1 | grep -v amdgpu.ids \
    | sed -E 's/"W": .*"linear": false, //' | cut -c1-90 | sed "s/^/round $k /" || exit 1
done
