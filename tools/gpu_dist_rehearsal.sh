# Rehearsal of bench.py's N > 1 path on a one-GPU box: 2 ranks over gloo,
# both rendering on the one GPU (RTW_SHARE_GPU).  The driver's N > 1 runs use
# RCCL with one rank per GPU; this exercises the rest of the multi-rank flow
# (row shards, barriers, max-over-ranks timing, gather to rank 0, one JSON line).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RTW_DIST_BACKEND=gloo RTW_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 \
  > gpurun_out/dist_rehearsal.json 2> gpurun_out/dist_rehearsal.err
