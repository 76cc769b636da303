#!/bin/bash
# Device ISA of the product variants only (var 0 / 8, mode 0) -> $OUT (default build/quick.s), then VGPR report.
# Extra hipcc flags as arguments (e.g. -DRTW_DEFAULT_VAR_F64=..., -gline-tables-only).
OUT=${OUT:-build/quick.s}
cd "$(dirname "$0")/../raytracinginoneweekend.zig_amd" && mkdir -p build &&
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-sched-strategy=iterative-ilp -I../include -Icsrc -DRTW_ISA_QUICK \
  --cuda-device-only -S csrc/rtw_trace.hip -o "$OUT" "$@" 2>&1 | grep -E "error" ; python ../tools/vgprs.py "$OUT"
