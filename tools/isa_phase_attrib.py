"""Static attribution of the megakernel's rotated loop (rtw_trace.hip, variant
with kVarMergedStart) to its PHASES: every VALU instruction of the loop and
of the loops nested in it is charged to the loop-body line of rtw_trace.hip
its inlined call chain starts from (the outermost `rtw_trace.hip:N` of the
instruction's .loc chain in a -gline-tables-only ISA dump), and the lines map
to the phases of the loop body: take units, sample start (u, v), the
cooperative sampler, scatter, camera ray, closest hit (bounce), finish.
Classes as tools/isa_attrib.py (f64, f32, int, cvt, "other").  Static counts:
an instruction of a nested loop counts once, whatever its trip count.

  python tools/isa_phase_attrib.py build/tqg.s 19826180"""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
path, var = sys.argv[1], sys.argv[2]
s = open(path).read()
src = open(__import__("os").path.join(__import__("os").path.dirname(__file__), "..", "raytracinginoneweekend.zig_amd",
                                      "csrc", "rtw_trace.hip")).read().split("\n")
# phase boundaries from the source: the rotated loop's statements
marks = {"take_units();": "take units", "start_sample_uv<R>(kargs<R>(), L, u, v);": "sample start (u, v)",
         "coop_reject_mixed<R>(dim": "cooperative sampler", "scatter_hit<R, F32, VAR, PRE>": "scatter",
         "start_sample_ray<R, PRE>": "camera ray", "const int b = bounce(kind, hit, tmax);": "closest hit (bounce)",
         "if (ended) finish_sample();": "finish sample"}
loop0 = next(i for i, l in enumerate(src) if "if constexpr ((VAR & kVarMergedStart) != 0) {" in l) + 1
loop1 = next(i for i, l in enumerate(src) if i > loop0 and l.strip() == "} else {") + 1
bounds = []
for i in range(loop0, loop1):
    for k, name in marks.items():
        if k in src[i - 1]:
            bounds.append((i, name))
bounds.sort()


def phase_of(line):
    if line is None or not (loop0 <= line <= loop1):
        return "other loop code"
    name = "loop control"
    for b, n in bounds:
        if line >= b:
            name = n
    return name


m = re.search(rf'^(_ZN4rtwk12trace_kernelIdLb\dELi0ELi{var}E\S*):', s, re.M)
body = s[m.end():s.find('.Lfunc_end', m.end())].split('\n')


def vclass(op):
    if re.search(r'_f64|_rcp_f64|_rsq_f64', op) and not op.startswith(('v_cmp', 'v_cvt')):
        return 'f64'
    if re.search(r'_f32|pk_', op) and not op.startswith(('v_cmp', 'v_cvt')):
        return 'f32'
    if op.startswith('v_cvt'):
        return 'cvt'
    if re.search(r'_u32|_i32|_u64|_i64|_u16|_b64', op) and re.search(r'(add|sub|mul|mad|lshl|ashr|lshr)', op):
        return 'int'
    return 'other'


# the hot loop: the header of the loop (depth 1) with the most VALU, and everything nested in it
hdr_valu = collections.Counter()
cur = None
for l in body:
    t = l.strip()
    if re.match(r'^\.LBB\d+_\d+:', t) or re.match(r'^; %bb\.\d+:', t):
        mm = re.search(r'Header=(BB\d+_\d+) Depth=1', t)
        cur = mm.group(1) if mm else None
        if 'Loop Header: Depth=1' in t:
            cur = t.split(':')[0].lstrip('.L')
        continue
    if cur and t.startswith('v_'):
        hdr_valu[cur] += 1
hot = hdr_valu.most_common(1)[0][0]
# loops nested in the hot one: headers whose label line names it as the depth-1 parent
inner = {hot}
for l in body:
    t = l.strip()
    mm = re.match(r'^\.L(BB\d+_\d+):\s*;\s*Parent Loop (BB\d+_\d+) Depth=1', t)
    if mm and mm.group(2) == hot:
        inner.add(mm.group(1))
cnt = collections.defaultdict(collections.Counter)
in_hot, line = False, None
for l in body:
    t = l.strip()
    if re.match(r'^\.LBB\d+_\d+:', t) or re.match(r'^; %bb\.\d+:', t):
        hm = re.search(r'Header=(BB\d+_\d+)', t)
        lab = re.match(r'^\.L(BB\d+_\d+):', t)
        in_hot = bool((hm and hm.group(1) in inner) or (lab and lab.group(1) in inner))
        continue
    mm = re.match(r'\.loc\s+\d+\s+\d+', t)
    if mm:
        chain = re.findall(r'rtw_trace\.hip:(\d+)', l)
        line = int(chain[-1]) if chain else None
        continue
    if in_hot and t.startswith('v_'):
        cnt[phase_of(line)][vclass(t.split()[0])] += 1
order = ["take units", "sample start (u, v)", "cooperative sampler", "scatter", "camera ray", "closest hit (bounce)",
         "finish sample", "loop control", "other loop code"]
tot = collections.Counter()
print(f"trace_kernel<d> var {var}: rotated loop {hot} and its nested loops, static VALU by phase and class")
print(f"{'phase':24s} {'all':>5s} {'f64':>5s} {'f32':>5s} {'int':>5s} {'cvt':>5s} {'other':>6s}")
for ph in order:
    c = cnt.get(ph)
    if not c:
        continue
    tot.update(c)
    print(f"{ph:24s} {sum(c.values()):5d} {c['f64']:5d} {c['f32']:5d} {c['int']:5d} {c['cvt']:5d} {c['other']:6d}")
print(f"{'total':24s} {sum(tot.values()):5d} {tot['f64']:5d} {tot['f32']:5d} {tot['int']:5d} {tot['cvt']:5d} {tot['other']:6d}")
