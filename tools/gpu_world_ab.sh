set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for occ in ${OCCS:-1 3 4}; do
  echo "occ $occ" >> gpurun_out/world_ab.log
  RTW_WORLD_OCC=$occ timeout -k 10 200 python tools/world_bench.py 6,7,1,3 >> gpurun_out/world_ab.log 2>&1 || exit 1
done
