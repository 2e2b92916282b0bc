#!/usr/bin/env python3
"""Instruction counts per basic block of one kernel in a hipcc -S listing
(tools/isa_count.py LISTING KERNEL_SUBSTRING)."""
import re
import sys

s = open(sys.argv[1]).read()
name = next(l.split(':')[0] for l in s.splitlines() if re.match(r'^_Z\S*' + sys.argv[2] + r'\S*:', l))
a = s.index(name + ':')
b = s.index('.Lfunc_end', a)
blocks, cur, cnt, kinds = [], 'entry', 0, {}
for l in s[a:b].splitlines()[1:]:
    t = l.strip()
    if re.match(r'^\.LBB\d+_\d+:', t) or t.startswith('; %bb'):
        blocks.append((cur, cnt, dict(kinds)))
        cur, cnt, kinds = t.split()[0] + (' loop' if 'Loop' in t else ''), 0, {}
    elif t and not t.startswith(';') and not t.startswith('.'):
        cnt += 1
        op = t.split()[0]
        k = 'v' if op.startswith('v_') else 's' if op.startswith('s_') else 'ds' if op.startswith('ds_') else 'mem'
        kinds[k] = kinds.get(k, 0) + 1
blocks.append((cur, cnt, kinds))
print(name[:90], 'total', sum(c for _, c, _ in blocks))
for n, c, k in blocks:
    print('%-24s %5d  %s' % (n, c, k))
