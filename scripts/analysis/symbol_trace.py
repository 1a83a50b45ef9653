# Analysis only (not product, not test): symbol-type traces (literal, matched
# literal, match, rep, short rep; decisions per symbol) of config-3 streams
# (lc0/lp0/pb0) from a plain-Python LZMA decode of liblzma output.
import sys, lzma, numpy as np, pickle
import os; R=os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0,os.path.join(R,'tests')); sys.path.insert(0,os.path.join(R,'lzma-sdk-zliblike_amd'))
import native
N=4096; COUNT=int(sys.argv[1]) if len(sys.argv)>1 else 128
plain=np.zeros(COUNT*N,dtype=np.uint8)
native.synth().synth_batch(0,0,plain.ctypes.data,N,COUNT,8)
filt=[{"id":lzma.FILTER_LZMA1,"dict_size":4096,"lc":0,"lp":0,"pb":0,"preset":6}]
def trace(buf):
    i=[5]; rng=0xFFFFFFFF; code=int.from_bytes(buf[1:5],'big')
    st=[rng,code]; probs={}
    cnt=[0,0]
    def bit(key):
        p=probs.get(key,1024)
        r,c=st
        if r<(1<<24): r=(r<<8)&0xFFFFFFFF; c=((c<<8)|buf[i[0]])&0xFFFFFFFF; i[0]+=1; cnt[1]+=1
        cnt[0]+=1
        b=(r>>11)*p
        if c<b: st[0]=b; st[1]=c; probs[key]=p+((2048-p)>>5); return 0
        st[0]=r-b; st[1]=c-b; probs[key]=p-(p>>5); return 1
    def direct():
        r,c=st
        if r<(1<<24): r=(r<<8)&0xFFFFFFFF; c=((c<<8)|buf[i[0]])&0xFFFFFFFF; i[0]+=1; cnt[1]+=1
        cnt[0]+=1
        r>>=1
        if c>=r: c-=r; st[0]=r; st[1]=c; return 1
        st[0]=r; st[1]=c; return 0
    def tree(pre,bits):
        m=1
        for _ in range(bits): m=(m<<1)|bit((pre,m))
        return m-(1<<bits)
    out=bytearray(); state=0; reps=[1,1,1,1]; syms=[]
    while len(out)<N:
        c0=list(cnt)
        if not bit(('M',state)):
            if state<7:
                sym=0x100|tree('L',8); kind='L'
            else:
                mb=out[-reps[0]]; offs=0x100; sym=1
                while sym<0x100:
                    mb<<=1; mbit=mb&offs
                    b=bit(('L',offs+mbit+sym)); sym=(sym<<1)|b
                    offs = (offs&mbit) if b else (offs&~mbit)
                kind='ML'
            out.append(sym&0xff); state = 0 if state<4 else (state-3 if state<10 else state-6)
            syms.append((kind,cnt[0]-c0[0],cnt[1]-c0[1],1)); continue
        if bit(('R',state)):
            if not bit(('G0',state)):
                if not bit(('R0L',state)):
                    state = 9 if state<7 else 11; out.append(out[-reps[0]])
                    syms.append(('SR',cnt[0]-c0[0],cnt[1]-c0[1],1)); continue
            else:
                if not bit(('G1',state)): d=reps[1]
                else:
                    if not bit(('G2',state)): d=reps[2]
                    else: d=reps[3]; reps[3]=reps[2]
                    reps[2]=reps[1]
                reps[1]=reps[0]; reps[0]=d
            lk='RL'; state = 8 if state<7 else 11; kind='REP'
        else:
            lk='LL'; reps[3]=reps[2]; reps[2]=reps[1]; reps[1]=reps[0]; state = 7 if state<7 else 10; kind='MA'
        if not bit((lk,'c')): ln=tree((lk,'lo'),3)
        elif not bit((lk,'c2')): ln=8+tree((lk,'mid'),3)
        else: ln=16+tree((lk,'hi'),8)
        if kind=='MA':
            slot=tree(('S',min(ln,3)),6)
            if slot<4: d=slot
            else:
                nb=(slot>>1)-1; d=(2|(slot&1))<<nb
                if slot<14:
                    m=1
                    for k in range(nb):
                        b=bit(('SP',d-slot,m)); m=(m<<1)|b; d|=b<<k
                else:
                    v=0
                    for k in range(nb-4): v=(v<<1)|direct()
                    d+=v<<4
                    m=1
                    for k in range(4):
                        b=bit(('A',m)); m=(m<<1)|b; d|=b<<k
            reps[0]=d+1
        ln+=2
        for _ in range(ln):
            if len(out)>=N: break
            out.append(out[-reps[0]])
        syms.append((kind,cnt[0]-c0[0],cnt[1]-c0[1],ln))
    return bytes(out), syms
T=[]
for s in range(COUNT):
    p=plain[s*N:(s+1)*N].tobytes()
    c=lzma.compress(p,format=lzma.FORMAT_RAW,filters=filt)
    o,syms=trace(b'\x00'*0+c)
    assert o==p, s
    T.append(syms)
pickle.dump(T,open('/tmp/lzgpu_traces.pkl','wb'))
from collections import Counter
C=Counter(); D=Counter()
for t in T:
    for k,d,nrm,ln in t: C[k]+=1; D[k]+=d
print({k:(C[k]/COUNT, D[k]/max(1,C[k])) for k in C})
