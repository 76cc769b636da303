# Wavefront shade_step with the merged cooperative pass (lib) vs the previous
# build (lib_o): wavefront GPU tests on lib (parity, exactly-once counts),
# then the frame A/B alternated in separate processes (tools/wf_bench.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_wf_merged.log 2>&1 &&
for r in 1 2 3; do
  for L in lib_o lib; do
    echo -n "lib=$L " >> gpurun_out/wf_merged_ab.txt
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/wf_bench.py 3 2>/dev/null >> gpurun_out/wf_merged_ab.txt || exit 1
  done
done
