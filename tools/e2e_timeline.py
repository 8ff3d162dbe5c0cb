"""Summarise traced end-to-end batches (tools/e2e_trace.py: gpurun_out/<tag>/trace.log):
pairs taken, last decode / retire, the dispatcher's issue() time, decode -> dispatch
delay, and the items in host decode per 10 ms.  Usage: python tools/e2e_timeline.py <tag> ..."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for tag in sys.argv[1:]:
    lines=open(os.path.join(ROOT, 'gpurun_out', tag, 'trace.log')).read().splitlines()
    mark=None; ev=[]
    for l in lines:
        if l.startswith('MARK'): mark=float(l.split()[1]); continue
        for m in re.finditer(r'\[zpx batch ([\d.]+)\] ([^\[]*)',l):
            if mark is not None and float(m.group(1))>=mark: ev.append((float(m.group(1))-mark, m.group(2).strip()))
    ev.sort(); t0=ev[0][0]
    dec={}; disp={}; ret={}; start={}; iss=[]; took={}; pairs=0
    for t,msg in ev:
        t-=t0
        m=re.match(r'worker: took item (\d+)( \+ (\d+))?',msg)
        if m:
            took[int(m.group(1))]=t
            if m.group(3) and m.group(3)!='-1': took[int(m.group(3))]=t; pairs+=1
        m=re.match(r'worker: item (\d+) fmt (\d) status \d+ decoded in ([\d.]+)s',msg)
        if m: dec[int(m.group(1))]=(t,int(m.group(2)))
        m=re.match(r'dispatch: item (\d+) -> slot',msg)
        if m: start[int(m.group(1))]=t
        m=re.match(r'dispatch: item (\d+) issued',msg)
        if m: disp[int(m.group(1))]=t; iss.append((int(m.group(1)), t-start[int(m.group(1))]))
        m=re.match(r'retire: item (\d+)',msg)
        if m: ret[int(m.group(1))]=t
    iss.sort(key=lambda x:-x[1])
    dl=[disp[i]-dec[i][0] for i in disp if i in dec]
    print(tag,'pairs',pairs,'last decode',round(max(v[0] for v in dec.values()),1),'last retire',round(max(ret.values()),1),
          'issue total',round(sum(x[1] for x in iss),1),'top',[(i,round(x,1)) for i,x in iss[:4]],
          'decode->dispatch mean',round(sum(dl)/len(dl),1),'max',round(max(dl),1))
    # worker-busy timeline: from took to decode end
    spans=[(took[i],dec[i][0]) for i in dec if i in took]
    row=''
    for q in range(0,int(max(ret.values()))+10,10):
        row+=f'{sum(1 for a,b in spans if a<=q<b):3d}'
    print('  items in decode per 10ms:',row)
