# A/B of the scheduler strategy for the world kernel and the wavefront engine:
# -mllvm -amdgpu-sched-strategy=max-memory-clause (lib_s3) / iterative-minreg (lib_s4) vs the default (lib).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
rm -f gpurun_out/ab_wf.txt gpurun_out/ab_world.txt
ENGINE=world LIBS="lib lib_s3 lib_s4" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null &&
ENGINE=wf LIBS="lib lib_s3 lib_s4" ROUNDS=2 bash tools/gpu_ab.sh > /dev/null &&
cat gpurun_out/ab_world.txt gpurun_out/ab_wf.txt | sed -E 's/"bvh.*"segments_per_sample"/"segments_per_sample"/'
