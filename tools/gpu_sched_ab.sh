# A/B of the LLVM AMDGPU scheduler strategy (whole library built with
# -mllvm -amdgpu-sched-strategy=max-ilp (lib_s1) / iterative-ilp (lib_s2) vs the default (lib)):
# megakernel, wavefront and world kernel timings, alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_mk.txt gpurun_out/ab_wf.txt gpurun_out/ab_world.txt
ENGINE=mk LIBS="lib lib_s1 lib_s2" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null &&
ENGINE=world LIBS="lib lib_s1 lib_s2" ROUNDS=2 bash tools/gpu_ab.sh > /dev/null &&
ENGINE=wf LIBS="lib lib_s1 lib_s2" ROUNDS=2 bash tools/gpu_ab.sh > /dev/null &&
cat gpurun_out/ab_mk.txt gpurun_out/ab_world.txt gpurun_out/ab_wf.txt
