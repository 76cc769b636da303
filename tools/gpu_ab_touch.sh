# World kernel A/B: each node visit also loads the first word of record node + 1 (the left child in
# the depth-first layout) with the node's record (lib_t, -DRTW_WORLD_TOUCH_NEXT=1), after the world
# GPU tests through it; then the globe's PMC passes through lib_t.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ENGINE=world LIBS="${LIBS:-lib lib_t}" TESTS="tests/test_gpu_world.py" ROUNDS=3 bash tools/gpu_ab.sh > /dev/null &&
RTW_LIB_PATH=raytracinginoneweekend.zig_amd/${PMCLIB:-lib_t}/librtw_hip.so SCENE=7 bash tools/gpu_world_pmc.sh &&
python tools/world_pmc_json.py gpurun_out 7 > gpurun_out/world_pmc_7_touch.json &&
cat gpurun_out/ab_world.txt
