# Analysis only (not product, not test): replays the symbol sequences written by
# symbol_trace.py through wave-scheduling policies of the literal batch and
# reports wave steps and lane efficiency per wave width.
import pickle, random, statistics
T=pickle.load(open('/tmp/lzgpu_traces.pkl','rb'))
LANES=16
def run(wave, policy, B=8, thr=0.5, ml_cost=8, match_extra=0):
    ptr=[0]*len(wave); steps=0.0
    live=lambda: [i for i in range(len(wave)) if ptr[i]<len(wave[i])]
    pend=[False]*len(wave)  # decoded IsMatch=1, waiting for match path
    while True:
        L=live()
        if not L: break
        # literal batch
        it=0
        while True:
            on=[i for i in L if not pend[i] and ptr[i]<len(wave[i])]
            if not on: break
            if policy=='batch' and it>=B: break
            if policy=='thr':
                if it>=B: break
                if it>0 and len(on) < thr*len(L): break
            steps+=1  # IsMatch
            kinds=set()
            for i in on:
                k=wave[i][ptr[i]][0]
                if k in ('L','ML'):
                    kinds.add(k); ptr[i]+=1
                else: pend[i]=True
            if 'L' in kinds: steps+=8
            if 'ML' in kinds: steps+=ml_cost
            it+=1
        mp=[i for i in L if pend[i]]
        if mp:
            ks=set(wave[i][ptr[i]][0] for i in mp)
            # match path: union of kinds; cost approx: rep bits 1-3, len ~4-5, slot+dist for MA
            c=1
            if 'MA' in ks: c+= 4 + 6 + 4 + match_extra
            if 'REP' in ks or 'SR' in ks: c+=3
            if 'REP' in ks: c+=4
            steps+=c
            for i in mp: ptr[i]+=1; pend[i]=False
    return steps
random.seed(1)
waves=[T[i:i+LANES] for i in range(0,len(T),LANES)]
useful=sum(sum(s[1] for s in t) for t in T)
for pol,args in [('batch',dict(B=8)),('batch',dict(B=4)),('batch',dict(B=16)),('batch',dict(B=1)),
                 ('thr',dict(B=8,thr=0.5)),('thr',dict(B=16,thr=0.5)),('thr',dict(B=32,thr=0.6)),('thr',dict(B=32,thr=0.4)),('thr',dict(B=64,thr=0.5)),('thr',dict(B=64,thr=0.7))]:
    tot=sum(run(w,pol,**args) for w in waves)
    print(pol,args, 'wave steps per wave %.0f'%(tot/len(waves)), 'lane eff %.3f'%(useful/(LANES*tot)))
print('--- lanes per wave')
for lanes in (8,16,32,64):
    ws=[T[i:i+lanes] for i in range(0,len(T),lanes)]
    for pol,args in [('batch',dict(B=8)),('thr',dict(B=32,thr=0.6))]:
        tot=sum(run(w,pol,**args) for w in ws)
        print(lanes,pol,args,'steps/wave %.0f'%(tot/len(ws)),'steps per 64 streams %.0f'%(tot/len(ws)*64/lanes), 'eff %.3f'%(useful/(lanes*tot)))
