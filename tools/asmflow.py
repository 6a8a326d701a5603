"""Compact control/memory flow of one kernel in an amdgcn .s file (dev helper).
Usage: python tools/asmflow.py file.s <mangled-name-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r'^(_Z\S*' + re.escape(sys.argv[2]) + r'\S*):', s, re.M)
name = names[0]
i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
out = [name, '\n']
for l in s[i:j].splitlines():
    if l.startswith('.LBB'):
        out.append('\n' + l.split(':')[0] + ': '); continue
    if not l.startswith('\t') or l.startswith('\t.') or l.startswith('\t;'):
        continue
    op = l.split()[0]
    if op.startswith('global_load'): out.append('G')
    elif op.startswith('global_store'): out.append('T')
    elif op.startswith('s_waitcnt'): out.append('[' + l.split(None, 1)[1].strip() + ']')
    elif op.startswith('ds_read'): out.append('r')
    elif op.startswith('ds_write'): out.append('w')
    elif 'fma' in op: out.append('f')
    elif op.startswith('s_cbranch') or op.startswith('s_branch'): out.append('B')
    elif op.startswith('scratch'): out.append('S')
print(''.join(out))
