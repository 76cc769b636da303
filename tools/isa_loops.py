"""Static VALU / SALU / LDS instruction counts per loop of one kernel in an ISA
dump (hipcc --cuda-device-only -S): for every loop header, the instructions of
the blocks LLVM labels as inside it (directly, not counting nested loops), so
two builds' hot loops can be compared before a GPU run.
Usage: isa_loops.py file.s kernel_regex"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(rf'^({sys.argv[2]}\S*):', s, re.M)
body = s[m.end():s.find('.Lfunc_end', m.end())].split('\n')
cnt = collections.defaultdict(lambda: [0, 0, 0])
cur = 'entry'
for l in body:
    t = l.strip()
    if re.match(r'^\.LBB\d+_\d+:', t):
        lab = t.split(':')[0]
        mm = re.search(r'Header=(BB\d+_\d+)', t)
        cur = ('.L' + mm.group(1)) if mm else (lab if 'Loop Header' in t else 'outside')
        continue
    if not t or t.startswith(('.', ';')):
        continue
    op = t.split()[0]
    c = cnt[cur]
    if op.startswith('v_'):
        c[0] += 1
    elif op.startswith('s_'):
        c[1] += 1
    elif op.startswith('ds_'):
        c[2] += 1
print(f"{'loop':14s} {'VALU':>6s} {'SALU':>6s} {'LDS':>5s}")
for k, (v, sa, d) in cnt.items():
    print(f"{k:14s} {v:6d} {sa:6d} {d:5d}")
