# wf_step register budget with 8 queue passes per launch: 6 waves/SIMD (lib_o6, spills 96 B) vs 5 (lib).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_wf.txt
ENGINE=wf LIBS="lib lib_o6" ROUNDS=4 bash tools/gpu_ab.sh > /dev/null && cat gpurun_out/ab_wf.txt
