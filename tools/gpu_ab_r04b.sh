# Round-4 A/B batch: megakernel xorshift from 32-bit ops (lib_x, -DRTW_XSH32=1) and the world
# kernel's node-visit case as one scalar word (lib_sd, -DRTW_WORLD_SCALAR_DECIDE=1), each
# after the GPU tests of its engine; then the globe's PMC passes through lib_sd.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ENGINE=mk LIBS="lib lib_x" TESTS="tests/test_gpu_parity.py tests/test_gpu_wavefront.py" ROUNDS=3 PMC="lib_x" \
  bash tools/gpu_ab.sh > /dev/null &&
ENGINE=world LIBS="lib lib_sd" TESTS="tests/test_gpu_world.py" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null &&
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/lib_sd/librtw_hip.so SCENE=7 bash tools/gpu_world_pmc.sh &&
cat gpurun_out/ab_mk.txt gpurun_out/ab_world.txt
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_clock.py \
  > gpurun_out/clock_test.txt 2>&1 && tail -3 gpurun_out/clock_test.txt &&
bash tools/gpu_dist_rehearsal.sh && python -c "import json;d=json.loads(open('gpurun_out/dist_rehearsal.json').read().strip().splitlines()[-1]);print(d['dist'], d['roofline'].get('evidence_scope'), d['roofline']['traffic'])"
