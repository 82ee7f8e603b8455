import re,collections,sys
SYM="_ZN3kgs12k_accumulateILi3EEEvPjS1_S1_PKjS3_jS3_jS1_"
L=open(sys.argv[1]).read().split('\n')
st=next(i for i,l in enumerate(L) if l.startswith(SYM+':'))
en=next(i for i in range(st,len(L)) if L[i].strip().startswith('.Lfunc_end'))
blocks=[];cur=('entry',[])
for l in L[st:en]:
    s=l.strip()
    if re.match(r'^\.LBB\d+_\d+:',s): blocks.append(cur);cur=(s.split(':')[0],[])
    elif s and not s.startswith(';') and not s.startswith('.'): cur[1].append(s)
blocks.append(cur)
hot=max(blocks,key=lambda b:len(b[1]))
c=collections.Counter(i.split()[0] for i in hot[1])
cost={'v_mad_u64_u32':4.16,'v_lshl_add_u64':4.4,'v_lshrrev_b64':4.16,'v_mul_lo_u32':4.28}
vop2=lambda op: op.endswith('_e32')
cyc=sum(v*(cost.get(k, 2.4 if vop2(k) else (1.0 if k.startswith('s_') else 4.2))) for k,v in c.items())
print(hot[0],len(hot[1]),'est cycles %.0f'%cyc)
for k,v in c.most_common(): print(f"  {k:28s}{v}")
m=[l for l in L[st:en] if 'vgpr_count' in l or 'NumVgprs' in l or 'ScratchSize' in l]
