#!/bin/bash
# Device ISA of the globe's world kernel only (world_kernel<0, 4, image|lane|packed>) -> $OUT
# (default build/world_q.s), then its VGPR / SGPR / scratch and scratch-instruction counts.
# Extra hipcc flags as arguments (e.g. -gline-tables-only).
OUT=${OUT:-build/world_q.s}
cd "$(dirname "$0")/../raytracinginoneweekend.zig_amd" && mkdir -p build &&
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc -DRTW_WORLD_ISA_QUICK \
  --cuda-device-only -S csrc/rtw_world.hip -o "$OUT" "$@" 2>&1 | grep -E "error"
grep -E "^\s+\.(private_segment_fixed_size|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count):" "$OUT"
echo "scratch stores: $(grep -c scratch_store "$OUT")  loads: $(grep -c scratch_load "$OUT")"
