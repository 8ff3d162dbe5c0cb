"""List s_waitcnt / VMEM ops of one kernel in a hipcc -S dump (ISA review aid)."""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
names = re.findall(r'^(\S*' + pat + r'\S*):', s, re.M)
k = names[0]
body = s[s.index(k + ':'):]
body = body[:body.index('.Lfunc_end')]
L = [l.strip() for l in body.split('\n')]
ins = [l for l in L if l and not l.startswith(('.', ';'))]
print(k, len(ins), 'instructions')
for i, l in enumerate(ins):
    if l.startswith('s_waitcnt') or 'buffer_load' in l or 'global_load' in l or l.endswith(':'):
        print(i, l[:110])
