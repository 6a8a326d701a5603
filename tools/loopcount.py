"""Instruction mix of the basic blocks holding >= 12 MFMAs of one kernel in an amdgcn .s file
(dev helper: the fused bins kernel's unrolled softmax / moment block).
Usage: python tools/loopcount.py file.s <mangled-name>"""
import collections
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
blocks, cur = [], None
for l in s[i:j].splitlines():
    if l.startswith('.LBB'):
        cur = [l.split(':')[0], []]
        blocks.append(cur)
        continue
    if cur is not None and l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'):
        cur[1].append(l.split()[0])
for bname, ins in blocks:
    if sum('mfma' in o for o in ins) < 12:
        continue
    c = collections.Counter()
    for o in ins:
        if 'mfma' in o: c['mfma'] += 1
        elif o.startswith('v_') and 'f64' in o: c['v_f64'] += 1
        elif o.startswith('v_'): c['v_other'] += 1
        elif o.startswith('ds_'): c['ds'] += 1
        elif o.startswith('s_'): c['s'] += 1
        else: c['other'] += 1
    print(bname, len(ins), dict(c))
    print('  other VALU:', collections.Counter(o for o in ins if o.startswith('v_') and 'f64' not in o).most_common(8))
    print('  f64 VALU:', collections.Counter(o for o in ins if o.startswith('v_') and 'f64' in o and 'mfma' not in o).most_common(8))
