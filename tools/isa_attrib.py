"""Static attribution of one trace_kernel instantiation's hot-loop VALU / SALU
instructions to source lines and instruction classes, from an ISA dump built
with -gline-tables-only (tools/isa_quick.sh -gline-tables-only, or make isa).
The classes follow the VALU mix of profiles/rNN/valu_issue.json: f64, f32 (and
packed f32), integer, conversion, and "other" (moves, selects, compares, bit and
lane operations: what the SQ counters do not split apart).

  python tools/isa_attrib.py build/quick_g.s d 19826180 [top] [loop-header]

The loop is the one with the most VALU instructions in its own blocks (nested
loops excluded, as tools/isa_loops.py) unless a header label is given."""
import collections
import re
import sys

path, prec, var = sys.argv[1], sys.argv[2], sys.argv[3]
top = int(sys.argv[4]) if len(sys.argv) > 4 else 25
want_hdr = sys.argv[5] if len(sys.argv) > 5 else None
s = open(path).read()
files = {}
for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s, re.M):
    files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
m = re.search(rf'^(_ZN4rtwk12trace_kernelI{prec}Lb\dELi0ELi{var}E\S*):', s, re.M)
body = s[m.end():s.find('.Lfunc_end', m.end())].split('\n')


def vclass(op):
    if not op.startswith('v_'):
        return None
    if re.search(r'_f64|_rcp_f64|_rsq_f64', op) and not op.startswith('v_cmp') and not op.startswith('v_cvt'):
        return 'f64'
    if op.startswith('v_cvt') or op.startswith('v_frexp') or op.startswith('v_ldexp'):
        return 'cvt'
    if op.startswith('v_cmp') or op.startswith('v_cndmask') or op.startswith('v_mov') or \
            re.match(r'v_(readlane|writelane|readfirstlane|mbcnt|bfrev|ffbh|ffbl|bcnt|perm|alignbit|alignbyte|bfi|'
                     r'bfe|and|or|xor|not|lshl|lshr|ashr|lshlrev|lshrrev|ashrrev|and_or|or3|xor3|lshl_or|'
                     r'lshl_add|add_lshl|max_u32|min_u32|max_i32|min_i32|swap|accvgpr)', op):
        return 'other'
    if re.search(r'_f32|_pk_', op) or op.startswith('v_pk'):
        return 'f32'
    return 'int'


# loop membership: a block belongs to the loop named in its "Loop Header"/"Header=" comment
blocks = []  # (loop, [(loc, op)])
cur_loop, cur = 'entry', []
loc = None
for l in body:
    t = l.strip()
    if re.match(r'^\.LBB\d+_\d+:', t):
        blocks.append((cur_loop, cur))
        lab = t.split(':')[0]
        mm = re.search(r'Header=(BB\d+_\d+)', t)
        cur_loop = ('.L' + mm.group(1)) if mm else (lab if 'Loop Header' in t else 'outside')
        cur = []
        continue
    mm = re.match(r'\.loc\s+(\d+)\s+(\d+)', t)
    if mm:
        loc = (files.get(mm.group(1)), int(mm.group(2)))
        continue
    if not t or t.startswith(('.', ';')):
        continue
    cur.append((loc, t.split()[0]))
blocks.append((cur_loop, cur))
per_loop = collections.Counter()
for lp, ins in blocks:
    per_loop[lp] += sum(1 for _, op in ins if op.startswith('v_'))
hdr = want_hdr or max((k for k in per_loop if k not in ('entry', 'outside')), key=lambda k: per_loop[k])
cls = collections.Counter()
by_line = collections.defaultdict(collections.Counter)
ops_other = collections.Counter()
salu = 0
for lp, ins in blocks:
    if lp != hdr:
        continue
    for lc, op in ins:
        if op.startswith('s_'):
            salu += 1
        c = vclass(op)
        if c is None:
            continue
        cls[c] += 1
        by_line[lc][c] += 1
        if c == 'other':
            ops_other[op.split('_e32')[0].split('_e64')[0]] += 1
tot = sum(cls.values())
print(f"trace_kernel<{prec}> var {var}: hot loop {hdr}: {tot} VALU, {salu} SALU (static, own blocks)")
print("classes:", ", ".join(f"{k} {v} ({100 * v / tot:.1f} %)" for k, v in cls.most_common()))
print("\"other\" by opcode:", ", ".join(f"{k} {v}" for k, v in ops_other.most_common(14)))
print(f"\ntop {top} source lines by \"other\" VALU (file:line  other / all VALU):")
for lc, c in sorted(by_line.items(), key=lambda kv: -kv[1]['other'])[:top]:
    print(f"  {lc[0] if lc else '?'}:{lc[1] if lc else '?'}  {c['other']} / {sum(c.values())}")
print(f"\ntop {top} source lines by all VALU:")
for lc, c in sorted(by_line.items(), key=lambda kv: -sum(kv[1].values()))[:top]:
    print(f"  {lc[0] if lc else '?'}:{lc[1] if lc else '?'}  {sum(c.values())}  " +
          " ".join(f"{k}={v}" for k, v in c.most_common()))
