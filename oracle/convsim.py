"""Encoder lane-convergence simulation on the spec model (oracle/spec.py,
diagnostics only): for lanes of S pairs started from the guessed state 2^L,
how many pairs until both chains meet the exact trajectory.  DESIGN.md section 5."""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import spec as S
def tables(data, L=None):
    counts, tl = None, None
    h = S.histogram(data)
    counts, size, tl = h if len(h)==3 else (h[0], len(data), h[1])
    if L is None: L = S.optimal_log2(len(data), tl)
    norm = S.normalize(counts, len(data), tl, L)
    if isinstance(norm, tuple): norm = norm[0]
    st, dnb, dfs = S.encode_table(norm, L, tl)
    return np.array(st, np.int64), np.array(dnb, np.int64), np.array(dfs, np.int64), L
def conv(kind, prob, L=None, nblk=4, T=64):
    out=[]
    for b in range(nblk):
        data = S.generate(kind, prob, 0x5EED0002, b, 65536)
        st,dnb,dfs,L2 = tables(data, L)
        n=len(data); P=n//2-1
        sym = np.frombuffer(data, np.uint8).astype(np.int64)
        # pairs p = P-1..0 : chain1 encodes sym[2p+1], chain0 sym[2p]
        Sl = P//T
        # true trajectory: run chains from exact init through all pairs, record state before pair p
        def step(x, s):
            nb = (dnb[s] + x) >> 16
            return st[(x >> nb) + dfs[s]]
        # exact init
        def init(s):
            bo=((dnb[s]+(1<<15))&0xffffffff)>>16; v=((bo<<16)-dnb[s])&0xffffffff
            return st[(v>>bo)+dfs[s]]
        x0=init(sym[n-2]); x1=init(sym[n-1])
        tr0=np.zeros(P+1,np.int64); tr1=np.zeros(P+1,np.int64)
        for p in range(P-1,-1,-1):
            tr0[p+1]=x0; tr1[p+1]=x1
            x1=step(x1,sym[2*p+1]); x0=step(x0,sym[2*p])
        tr0[0]=x0; tr1[0]=x1
        # boundaries: lane k range [k*Sl,(k+1)*Sl), starts at pair (k+1)*Sl-1 with state tr[(k+1)*Sl]
        ks=np.arange(T-1)
        tops=(ks+1)*Sl
        y0=np.full(T-1,1<<L2); y1=np.full(T-1,1<<L2)
        d=np.full(T-1,-1)
        for t in range(Sl):
            p=tops-1-t
            m=(y0==tr0[p+1])&(y1==tr1[p+1])&(d<0)
            d[m]=t
            y1=step(y1,sym[2*p+1]); y0=step(y0,sym[2*p])
        m=(y0==tr0[tops-Sl])&(y1==tr1[tops-Sl])&(d<0); d[m]=Sl
        out.append(d)
    d=np.concatenate(out)
    nc=(d<0).sum()
    dd=d[d>=0]
    print(f"kind={kind} p={prob} T={T} S={Sl}: never {nc}/{len(d)}  mean {dd.mean():.0f} p50 {np.median(dd):.0f} p90 {np.percentile(dd,90):.0f} max {dd.max()}  per-block max {[int(x.max()) for x in out]}")
conv(0,0.155)
conv(2,0.0,11)
conv(0,0.77,11,nblk=2)
conv(0,0.155,T=32)
