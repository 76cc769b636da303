# Round-3 checkpoint: every GPU test + smoke (current build), megakernel A/B
# lib_o (round 2) vs lib, the VALU PMC of lib, and the survivor-loop
# duplication measurement (lib vs lib_dup timing, VALU PMC of lib_dup).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ENGINES="mk" ROUNDS=3 bash tools/gpu_r03_step.sh &&
TAG=r03v bash tools/gpu_pmc_valu.sh &&
bash tools/gpu_r03_step3.sh
