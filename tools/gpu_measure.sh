# Phase-duplication measurement (RTW_MEASURE build): time A/B of the
# variants and SQ_INSTS_VALU per variant (one PMC pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=${V:-516,2564,4612,8708,16900}
timeout -k 10 400 python tools/ab_variants.py f64 $V 4 > gpurun_out/measure_ab.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/measure_pmc -o run \
  --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_VALU \
  -- python tools/measure_run.py f64 $V > gpurun_out/measure_pmc.log 2>&1
