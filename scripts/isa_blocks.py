"""Basic-block instruction counts of one kernel in a gfx950 .s file (dev tool).
usage: python scripts/isa_blocks.py file.s <mangled-name-substring> [min_instrs]"""
import re
import sys

s = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 0
a = next(i for i, l in enumerate(s) if re.match(r'^_Z\S*' + re.escape(pat) + r'\S*:', l))
b = next(i for i in range(a, len(s)) if s[i].startswith('.Lfunc_end'))
blocks, cur = [], ['entry', 0, 0, 0, []]
blocks.append(cur)
for l in s[a:b]:
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        cur = [m.group(1), 0, 0, 0, []]
        blocks.append(cur)
        continue
    if l.startswith('\t') and not l.strip().startswith(('.', ';')):
        op = l.split()[0]
        cur[1] += 1
        cur[2] += op.startswith('v_')
        cur[3] += op.startswith('s_')
        if 'load' in op or 'store' in op or op.startswith('ds_') or 'branch' in op or 'swappc' in op:
            cur[4].append(op.replace('global_', 'g_').replace('s_cbranch_', 'br_'))
tot = sum(x[1] for x in blocks)
print(f"{pat}: {tot} instrs in {len(blocks)} blocks")
for x in blocks:
    if x[1] >= mn:
        print(f"{x[0]:12s} n{x[1]:4d} v{x[2]:4d} s{x[3]:4d} | {' '.join(x[4])[:150]}")
