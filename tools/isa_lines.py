"""Static per-source-line counts of chosen instructions in one trace_kernel
instantiation of an ISA dump built with -gline-tables-only.
Usage: isa_lines.py file.s <prec d|f> <var> <regex> [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
prec, var, pat = sys.argv[2], sys.argv[3], re.compile(sys.argv[4])
top = int(sys.argv[5]) if len(sys.argv) > 5 else 30
files = {}
for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s, re.M):
    files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
m = re.search(rf'^(_ZN4rtwk12trace_kernelI{prec}Lb\dELi0ELi{var}E\S*):', s, re.M)
body = s[m.end():s.find('.Lfunc_end', m.end())].split('\n')
cur, cnt = None, collections.Counter()
for l in body:
    t = l.strip()
    mm = re.match(r'\.loc\s+(\d+)\s+(\d+)', t)
    if mm:
        cur = (files.get(mm.group(1)), int(mm.group(2)))
        continue
    if pat.match(t):
        cnt[cur] += 1
print('total', sum(cnt.values()))
for k, v in cnt.most_common(top):
    print(v, k)
