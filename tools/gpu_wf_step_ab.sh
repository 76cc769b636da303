# wf_step register target (lib: 4 waves/SIMD, lib_s5: 5) x queue capacity
# (tools/wf_sweep.py), builds alternated in separate processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
for r in 1 2; do
  for L in lib lib_s5; do
    echo "lib $L" >> gpurun_out/wf_step_ab.txt
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 300 python tools/wf_sweep.py f64 1048576,1572864,2097152 \
      >> gpurun_out/wf_step_ab.txt 2>> gpurun_out/wf_step_ab.err || exit 1
  done
done
