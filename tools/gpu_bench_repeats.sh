#!/bin/bash
# The bench line's run-to-run spread on one box: python bench.py (defaults, --no-cpu-baseline) N times
# in separate processes; one summary line per run (headline, f32, wavefront + its HBM frac, globe, Cornell).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bench_repeats.txt
for i in $(seq 1 ${N:-3}); do
  timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_rep_$i.json 2> gpurun_out/bench_rep_$i.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/bench_rep_$i.json')); w=d['wavefront_variant']
print('run $i', d['value'], d['roofline']['frac'], d['roofline']['sclk_mhz'], d['f32_hybrid_variant']['value'], w['value'],
      w['roofline']['frac'], d['globe_10k_variant']['value'], d['cornell_variant']['value'])" >> gpurun_out/bench_repeats.txt
done
cat gpurun_out/bench_repeats.txt
