# Round 3: the new full-workload oracle tests (configs[4] globe rows, full
# Cornell frame, clustered pretest with mixed time groups), the megakernel /
# wavefront parity tests (coop sampler change), then the gloo rehearsal of
# bench.py --gpus 2 (per-rank timing fields) and one bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py" \
  "tests/test_gpu_world.py::test_cornell_full_frame_equals_oracle" \
  "tests/test_gpu_world.py::test_globe_config4_workload_equals_oracle" > gpurun_out/r03_newtests.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_bench1.json 2> gpurun_out/r03_bench1.err &&
RTW_DIST_BACKEND=gloo RTW_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-world-variants > gpurun_out/dist_rehearsal.json 2> gpurun_out/dist_rehearsal.err
