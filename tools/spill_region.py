#!/usr/bin/env python3
"""Spill instructions (scratch_*, v_readlane/v_writelane) of one kernel in a hipcc -S -gline-tables-only
assembly whose inline chain touches source lines [lo, hi].  usage: spill_region.py <asm> <kernel substring> <lo> <hi>"""
import re,sys,collections
f,fn,lo,hi=sys.argv[1],sys.argv[2],int(sys.argv[3]),int(sys.argv[4])
lines=open(f).read().split('\n')
st=next(i for i,l in enumerate(lines) if l.startswith("_Z") and fn in l.split(":")[0])
en=st
while not lines[en].startswith(".Lfunc_end"): en+=1
cur=0; inl=""
res=[]
for j in range(st,en):
    l=lines[j].strip()
    m=re.match(r"\.loc\s+\d+\s+(\d+).*?;\s*(\S+)",l)
    if m:
        ln=int(m.group(1))
        if ln: cur=ln; inl=l.split(';',1)[1].strip()
        continue
    if re.match(r"(scratch_|v_readlane|v_writelane)",l):
        # find the outermost routes.hip line in the inline chain
        chain=[int(x) for x in re.findall(r"routes(?:_orig)?\.hip:(\d+)",inl)]
        if any(lo<=c<=hi for c in chain):
            res.append((j-st,l.split(';')[0].strip(),chain[:4]))
for r in res: print(r)
print(len(res))
