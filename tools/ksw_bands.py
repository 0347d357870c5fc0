"""Band shape of ksw_extend2 (software/ksw.c:379-476) on problems shaped like
mem_chain2aln's (synth.make_ksw_tasks), by a plain restatement of the row loop
that records each row's band [beg, end): the fraction of a query a row's band
covers and of 8-column chunks fully inside it -- why the lane engine's chunks
mostly run masked.  CPU only.

    python tools/ksw_bands.py [--problems 300] [--min-qlen 65] [--max-qlen 128]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from smemgpu import synth
g = synth.make_genome(2_000_000, seed=771, n_chrom=1)
kb = synth.make_ksw_tasks(g.codes, 3000, seed=771)
mat = np.array(kb.mat, dtype=np.int64).reshape(5,5) if hasattr(kb,'mat') else None
o_del,e_del,o_ins,e_ins = 6,1,6,1
def ext(q, t, w, end_bonus, zdrop, h0):
    qlen=len(q); tlen=len(t)
    oe_del=o_del+e_del; oe_ins=o_ins+e_ins
    h=[0]*(qlen+1); e=[0]*(qlen+1)
    h[0]=max(h0,0); h0=max(h0,0)
    h[1]=h0-oe_ins if h0>oe_ins else 0
    j=2
    while j<=qlen and h[j-1]>e_ins: h[j]=h[j-1]-e_ins; j+=1
    top=1
    mi=int((qlen*top+end_bonus-o_ins)/e_ins+1.); mi=max(mi,1); w=min(w,mi)
    md=int((qlen*top+end_bonus-o_del)/e_del+1.); md=max(md,1); w=min(w,md)
    mx=h0; max_i=max_j=-1; beg=0; end=qlen; bands=[]
    for i in range(tlen):
        f=0; m=0; mj=-1
        h1=max(h0-(o_del+e_del*(i+1)),0)
        if beg<i-w: beg=i-w
        if end>i+w+1: end=i+w+1
        if end>qlen: end=qlen
        bands.append((beg,end))
        for jj in range(beg,end):
            M=h[jj]; E=e[jj]; h[jj]=h1
            M+=mat[t[i]][q[jj]]
            H=max(M,E,f); h1=H
            if H>=m: mj=jj; m=H  # m>h?mj:j
            tt=max(H-oe_del,0); E=max(E-e_del,tt); e[jj]=E
            tt=max(H-oe_ins,0); f=max(f-e_ins,tt)
        h[end]=h1; e[end]=0
        if m==0: break
        if m>mx: mx=m; max_i=i; max_j=mj
        elif zdrop>0:
            if i-max_i>mj-max_j:
                if mx-m-((i-max_i)-(mj-max_j))*e_del>zdrop: break
            elif mx-m-((mj-max_j)-(i-max_i))*e_ins>zdrop: break
        jj=mj
        while jj>=beg and h[jj]: jj-=1
        beg=jj+1
        jj=mj+2
        while jj<=end and h[jj]: jj+=1
        end=jj
    return bands
tot=0; full=0; rows=0; cover=0
ap = argparse.ArgumentParser()
ap.add_argument("--problems", type=int, default=300)
ap.add_argument("--min-qlen", type=int, default=65)
ap.add_argument("--max-qlen", type=int, default=128)
a = ap.parse_args()
sel=[k for k in range(kb.tasks.size) if a.min_qlen<=kb.tasks['qlen'][k]<=a.max_qlen]
for k in sel[:a.problems]:
    T=kb.tasks[k]
    qo=int(T['q_off']); to=int(T['t_off']); q=kb.q[qo:qo+int(T['qlen'])]; t=kb.t[to:to+int(T['tlen'])]
    b=ext(list(q),list(t),int(T['w']),int(T['end_bonus']),int(T['zdrop']),int(T['h0']))
    ql=int(T['qlen'])
    for (bg,en) in b:
        rows+=1
        for c in range((ql+7)//8):
            tot+=1
            if bg<=8*c and en>=8*c+8: full+=1
        cover+=max(en-bg,0)/ql
print('problems',len(sel[:a.problems]),'rows',rows,'chunk fraction full per lane',full/tot,'mean band/qlen',cover/rows)
