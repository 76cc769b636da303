# Round-5 A/B of the Tier-B mixer (RTW_RNG_MIX): lib = Feistel x4 (mixer 10, the new
# contract), lib_m0 = SplitMix64 (rounds 1-4), lib_m1 = its 32-bit-fold form, lib_m2 = one
# multiply between two folds (fails tests/native/rng_stats.c; speed only). Images differ
# between builds, so this is timing only: megakernel (configs[1] f64 + f32), wavefront
# (configs[3]), world kernel (globe configs[4] + Cornell).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ENGINE=mk LIBS="lib_m0 lib_m1 lib_m2 lib" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null &&
ENGINE=wf LIBS="lib_m0 lib" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null &&
ENGINE=world LIBS="lib_m0 lib" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null &&
cat gpurun_out/ab_mk.txt gpurun_out/ab_wf.txt gpurun_out/ab_world.txt
