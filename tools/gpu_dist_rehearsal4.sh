# bench.py's N > 1 path with 4 ranks on the one-GPU box (gloo, all ranks on the card; the driver's
# N > 1 runs use RCCL with one rank per GPU): row shards, barriers, max-over-ranks timing, gather.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RTW_DIST_BACKEND=gloo RTW_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 6 --warmup 2 \
  --no-cpu-baseline --no-wavefront-variant --no-world-variants --no-f32-variant \
  > gpurun_out/dist_rehearsal4.json 2> gpurun_out/dist_rehearsal4.err && tail -c 700 gpurun_out/dist_rehearsal4.json
