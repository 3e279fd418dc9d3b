#!/usr/bin/env python3
"""Division digit study (CPU only, diagnostic, round 6): for DIV nodes of the bench's synthetic
states, per 64-candidate wave (candidates drawn as 25 % interesting / 75 % uniform values), how
many waves take the single-digit path of the gfx950 interpreter's DIV, how many Knuth digits the
others run (max over dividing lanes of top limb(a) - top limb(b), + 1), and the same with the
one-limb-divisor lanes left out (what a short-division path for those lanes would leave).
    python profiles/div_digits.py [n_states]  -> profiles/div_digits_r6.txt"""
import sys, collections
sys.path.insert(0,'/root/repo')
import numpy as np
from mythril_amd import _native as N
from oracle import bvsem as S
from tests._util import state_slice
SEED=0x4D595448
ns=int(sys.argv[1]) if len(sys.argv)>1 else 128
b = N.synth_generate(SEED, 0, ns, 64, 256)
rng = np.random.default_rng(0)
# candidates: use the device fill kernel? not available on CPU; approximate with host mixture
# reuse make-like mixture: 25% interesting, 75% uniform
INTER=[0,1,(1<<256)-1,1<<255,(1<<160)-1,0xDEADBEEF*((1<<160)-1)//0xFFFFFFFF]
stats=collections.Counter()
digits=[]; digits2=[]
for s in range(ns):
    nodes, consts = state_slice(b, s)
    nv = b["n_vars"]
    divs=[i for i,n in enumerate(nodes) if int(n["op"]) in (S.UDIV,S.UREM,S.SDIV,S.SREM)]
    if not divs: continue
    for chunk in range(4):
        ks=[]; single=True; dmax=-1
        tops_b=[]
        for lane in range(64):
            xs=[ (INTER[rng.integers(len(INTER))] if rng.random()<0.25 else int.from_bytes(rng.bytes(32),'little')) for _ in range(nv)]
            vals=S.eval_dag(nodes, consts, xs)
            ks.append(vals)
        for di in divs:
            n=nodes[di]
            dmax=-1; single=True; smallb=0; dmax2=-1; single2=True
            for vals in ks:
                a=vals[int(n["a"])] & ((1<<256)-1); bb=vals[int(n["b"])] & ((1<<256)-1)
                if int(n["op"]) in (S.SDIV,S.SREM):
                    if a>>255: a=(1<<256)-a
                    if bb>>255: bb=(1<<256)-bb
                if bb==0 or a<bb: continue
                if (a>>32) >= bb: single=False
                ta=(a.bit_length()-1)//32; tb=(bb.bit_length()-1)//32
                dmax=max(dmax, ta-tb)
                if tb==0: smallb+=1
                elif (a>>32) >= bb: single2=False; dmax2=max(dmax2, ta-tb)
            stats['single' if single else 'multi']+=1
            if not single: digits.append(dmax+1)
            if not single: digits2.append((smallb>0, 'single' if single2 else dmax2+1))
            stats[('smallb_lanes>0', smallb>0)]+=1
print(stats)
print(collections.Counter(digits)); print(sorted(collections.Counter(digits2).items(), key=str))
