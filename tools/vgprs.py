"""Print VGPR / SGPR / scratch of each trace_kernel instantiation (make isa first)."""
import re
import sys

s = open(sys.argv[1] if len(sys.argv) > 1 else "build/rtw_trace-gfx950.s").read()
for blk in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
    name, b = blk.group(1), blk.group(2)
    m = re.search(r"trace_kernelI([df])Lb\dELi(\d)ELi(\d+)E", name)
    if not m or m.group(2) != "0":
        continue
    g = lambda k: re.search(k + r" (\d+)", b).group(1)
    print(f"{'f64' if m.group(1) == 'd' else 'f32'} var{m.group(3):>3}: vgpr {g('amdhsa_next_free_vgpr')} "
          f"sgpr {g('amdhsa_next_free_sgpr')} scratch {g('amdhsa_private_segment_fixed_size')}")
