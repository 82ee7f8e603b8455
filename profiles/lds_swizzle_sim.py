#!/usr/bin/env python3
"""LDS bank-conflict model of the NTT LDS passes (k_ntt_lds_pass): for every access pattern of a pass
(address-order staging in the contiguous / run-wise layouts, each register round), the mean and worst
number of 16-byte slots per bank group in a 16-lane phase of ds_read/write_b128, for candidate slot
swizzles. usage: python profiles/lds_swizzle_sim.py"""
import itertools
ELOG=11; NT=256
def patterns(K, R3, dit):
    LBLOG=ELOG-K; LB=1<<LBLOG
    pats=[]
    # staged (contiguous: logd=0): e -> j = e & (2^K-1), cl = e >> K
    for k in range((1<<ELOG)//NT):
        pats.append([ ((e & ((1<<K)-1))*LB + (e>>K)) for e in range(k*NT, k*NT+NT)])
    rs = [3,3,R3] if R3 else [3,3]
    Ks=[r for r in rs]
    # b0 per round
    if dit:
        b0s=[0, rs[0], rs[0]+rs[1]][:len(rs)]
    else:
        b0s=[K-rs[0], K-rs[0]-rs[1], 0][:len(rs)] if len(rs)==3 else [K-rs[0], 0]
    for R,b0 in zip(rs,b0s):
        ng=(1<<ELOG)>>R
        for it in range(ng//NT):
            for r in range(1<<R):
                sl=[]
                for g in range(it*NT, it*NT+NT):
                    cl=g&(LB-1); jq=g>>LBLOG
                    jb=(jq & ((1<<b0)-1)) | ((jq>>b0)<<(b0+R))
                    sl.append((jb+(1<<b0)*r)*LB+cl)
                pats.append(sl)
    return pats
def cost(pats, sw):
    tot=0; worst=0
    for p in pats:
        for w in range(0,NT,64):
            for g in range(w, w+64, 16):
                c={}
                for s in p[g:g+16]:
                    b=sw(s)%16; c[b]=c.get(b,0)+1
                m=max(c.values()); tot+=m; worst=max(worst,m)
    return tot/(len(pats)*NT/16), worst
cands={'none':lambda s:s}
for sh in range(2,9):
    for mbits in (2,3,4):
        cands[f'x>>{sh}&{(1<<mbits)-1}']=(lambda sh,m: (lambda s: s ^ ((s>>sh)&m)))(sh,(1<<mbits)-1)
cands['x>>4^x>>8']=lambda s: s ^ ((s>>4)&15) ^ ((s>>8)&15)
cands['x>>2^x>>6']=lambda s: s ^ ((s>>2)&3) ^ (((s>>6)&3)<<2)
for (K,R3) in ((9,3),(8,2),(7,2),(6,0),(5,0)):
    for dit in (False,True):
        if (K,R3)==(5,0): rs=None
        pats=patterns(K,R3,dit) if K>=6 else None
        if pats is None: continue
        res=sorted(((cost(pats,f),n) for n,f in cands.items()))
        base=cost(pats,cands['none'])
        print(K,R3,'DIT' if dit else 'DIF','none',base,'best',res[:4])
print('--- runs mode (non-contiguous passes): rounds + consecutive staged')
def patterns_runs(K,R3,dit):
    p=patterns(K,R3,dit)
    nst=(1<<ELOG)//NT
    return [list(range(k*NT,k*NT+NT)) for k in range(nst)] + p[nst:]
for name in ('none','x>>4&15','x>>4^x>>8','x>>3&15','x>>5&15'):
    row=[]
    for (K,R3) in ((9,3),(8,2),(7,2),(6,0)):
        for dit in (False,True):
            a=cost(patterns(K,R3,dit),cands[name])[0]; b=cost(patterns_runs(K,R3,dit),cands[name])[0]
            row.append(f'{K}{"T" if dit else "F"}:{a:.2f}/{b:.2f}')
    print(name.ljust(10),' '.join(row))
