"""Rough check that every register loaded by a buffer_load/global_load in a
kernel is not read before an s_waitcnt vmcnt(N) that covers it (linear code
order, with one wrap-around for the step loop's back-edge).  ISA review aid
for the hand-counted waits in png_kernels.hip."""
import re
import sys

s = open(sys.argv[1]).read()
k = re.findall(r'^(\S*' + sys.argv[2] + r'\S*):', s, re.M)[0]
body = s[s.index(k + ':'):]
body = body[:body.index('.Lfunc_end')]
ins = [l.strip() for l in body.split('\n') if l.strip() and not l.strip().startswith(('.', ';'))]


def regs(tok):
    m = re.match(r'v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)$', tok)
    return {int(m.group(1))} if m else set()


def operands(l):
    parts = l.split(None, 1)
    if len(parts) < 2:
        return parts[0], []
    return parts[0], [t.strip() for t in parts[1].split(',')]


bad = 0
n = len(ins)
for i, l in enumerate(ins):
    op, ops = operands(l)
    if not (op.startswith('buffer_load') or op.startswith('global_load')):
        continue
    dst = regs(ops[0])
    loads_after = 0
    covered = False
    for j in range(1, 2 * n):
        l2 = ins[(i + j) % n]
        op2, ops2 = operands(l2)
        if op2 == 's_waitcnt':
            m = re.search(r'vmcnt\((\d+)\)', l2)
            if m and int(m.group(1)) <= loads_after:
                covered = True
                break
            continue
        src = set()
        for t in ops2[1:] if not op2.startswith(('global_store', 'buffer_store')) else ops2:
            src |= regs(t)
        if op2.startswith(('buffer_load', 'global_load')):
            loads_after += 1
            src = set()
            for t in ops2[1:]:
                src |= regs(t)
        if src & dst:
            print('UNCOVERED read of', ops[0], 'loaded at', i, ':', l[:60], '-> read at', (i + j) % n, ':', l2[:80])
            bad += 1
            break
        # a redefinition (not a read) of all dst regs ends the live range
        if ops2 and regs(ops2[0]) >= dst and not op2.startswith(('global_store', 'buffer_store', 's_')):
            break
print(k[:60], 'loads checked; uncovered reads:', bad)
sys.exit(1 if bad else 0)
