# A/B: the megakernel's loop-carried ray state pinned at the loop top by an empty asm
# (RTW_LANE_PIN=1: o, d, T, time; =9: also rs, tmax, hit, kind, depth, s, skip) vs none (lib).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_mk.txt
ENGINE=mk LIBS="lib lib_p1 lib_p9" ROUNDS=4 bash tools/gpu_ab.sh > /dev/null && cat gpurun_out/ab_mk.txt
