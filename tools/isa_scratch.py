"""Where one kernel's scratch (spill) instructions sit: for every scratch_load /
scratch_store, its loop (LLVM's block comment: header and depth) and, from a
-gline-tables-only dump, the source line.  Per loop depth, the count.
Usage: isa_scratch.py file.s kernel_regex"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(rf'^({sys.argv[2]}\S*):', s, re.M)
files = dict(re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s, re.M))
body = s[m.end():s.find('.Lfunc_end', m.end())].split('\n')
loop, depth, loc = 'entry', 0, None
per = collections.Counter()
for l in body:
    t = l.strip()
    mm = re.match(r'^\.LBB\d+_\d+:', t) or re.match(r'^; %bb\.\d+:', t)
    if mm:
        h = re.search(r'Header=(BB\d+_\d+) Depth=(\d+)', t)
        if h:
            loop, depth = h.group(1), int(h.group(2))
        elif 'Loop Header' in t:
            d = re.search(r'Depth=(\d+)', t)
            loop, depth = t.split(':')[0], int(d.group(1)) if d else 1
        else:
            loop, depth = 'outside', 0
        continue
    lc = re.match(r'\.loc\s+(\d+)\s+(\d+)', t)
    if lc:
        loc = f"{files.get(lc.group(1), lc.group(1)).split('/')[-1]}:{lc.group(2)}"
        continue
    if t.startswith('scratch_'):
        per[depth] += 1
        print(f"depth {depth} {loop:12s} {loc or '':24s} {t[:60]}")
print('per loop depth:', dict(sorted(per.items())))
