# The round's evidence from ONE box, in order: every GPU test + smoke(); the PMC passes the bench
# line reads (trace VALU issue + traffic, wavefront traffic, world kernel globe + Cornell),
# converted to JSON and written both to profiles/$TAG/ of this box's copy (so the bench line
# below reads them) and to gpurun_out/ev/ (copied back into the repo); the bench line and the
# rocprofv3 kernel statistics of the same command; configs[2] (3840x2160x2000) on this one GPU
# with its kernel statistics (the strong-scaling T(1)); the 2-rank gloo rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp RTW_WF_TIMEOUT_S=60
TAG=${TAG:-r06}
mkdir -p gpurun_out/ev profiles/$TAG
ev() { cp "$1" profiles/$TAG/ && cp "$1" gpurun_out/ev/; }
bash tools/gpu_tests.sh &&
TAG=${TAG}v bash tools/gpu_pmc_valu.sh &&
python tools/valu_json.py gpurun_out/${TAG}v_a gpurun_out/${TAG}v_b gpurun_out/${TAG}v_c gpurun_out/valu_issue.json > /dev/null &&
ev gpurun_out/valu_issue.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_fetch -o run \
  --pmc FETCH_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_${TAG}_write -o run \
  --pmc WRITE_SIZE -- python tools/prof_run.py f64 > gpurun_out/pmc_write.log 2>&1 &&
python tools/traffic_json.py gpurun_out/pmc_${TAG}_fetch gpurun_out/pmc_${TAG}_write gpurun_out/traffic.json > /dev/null &&
ev gpurun_out/traffic.json &&
bash tools/gpu_pmc_wf.sh > /dev/null && ev gpurun_out/wf_traffic.json &&
python tools/wf_kernel_pmc.py gpurun_out/wf_issue_a gpurun_out/wf_issue_b > gpurun_out/ev/wf_issue.txt &&
bash tools/gpu_world_pmc_both.sh && ev gpurun_out/world_pmc_7.json && ev gpurun_out/world_pmc_6.json &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run \
  -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 &&
timeout -k 10 600 python bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline --no-wavefront-variant \
  --no-world-variants --no-f32-variant > gpurun_out/bench_config2.json 2> gpurun_out/bench_config2.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_c2 -o run \
  -- python bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline --no-wavefront-variant --no-world-variants \
  --no-f32-variant > gpurun_out/bench_config2_prof.log 2>&1 &&
bash tools/gpu_dist_rehearsal.sh &&
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['wavefront_variant']['value'], d['globe_10k_variant']['value'], d['cornell_variant']['value'], d['cpu_baseline']['value'])"
