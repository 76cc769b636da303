# PMC passes over the world kernel (scene $SCENE): issue/wait breakdown, I-cache, instruction mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${SCENE:-6}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wpmc_${S}_a -o run \
  --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
  -- python tools/world_prof_run.py $S > gpurun_out/wpmc_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wpmc_${S}_b -o run \
  --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA \
  -- python tools/world_prof_run.py $S > gpurun_out/wpmc_b.log 2>&1
