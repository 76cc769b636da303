# Queue capacity sweep (wf_paths) for builds in LIBS: segment counts that are
# whole multiples of the extend / shade persistent wave counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
mkdir -p gpurun_out
P=raytracinginoneweekend.zig_amd
for r in 1 2; do
  for L in ${LIBS:-lib}; do
    echo "lib $L" >> gpurun_out/wf_sweep3.txt
    RTW_LIB_PATH=$P/$L/librtw_hip.so timeout -k 10 300 python tools/wf_sweep.py f64 ${PATHS:-786432,1048576,1179648,1572864,2097152} \
      >> gpurun_out/wf_sweep3.txt 2>> gpurun_out/wf_sweep3.err || exit 1
  done
done
