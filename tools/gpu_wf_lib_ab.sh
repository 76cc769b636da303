# Wavefront engine A/B of two builds (lib vs lib_c, RTW_LIB_PATH), after the
# wavefront GPU tests; alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_wavefront.py -x -q --timeout 300 > gpurun_out/pytest_wf.log 2>&1 &&
for r in 1 2 3; do
  for L in lib lib_c; do
    echo -n "$L " >> gpurun_out/wf_ab.log
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 200 python tools/wf_bench.py 3 2>/dev/null >> gpurun_out/wf_ab.log || exit 1
  done
done
