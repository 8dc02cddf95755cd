import numpy as np
rng=np.random.default_rng(0)
def bf16(x):
    x=np.asarray(x,np.float32); b=x.view(np.uint32).astype(np.uint64)
    r=((b+0x7fff+((b>>16)&1))>>16)<<16
    return r.astype(np.uint32).view(np.float32)
def f16(x): return np.asarray(x,np.float32).astype(np.float16).astype(np.float32)
K=256; M=64; N=2000
A=(rng.standard_normal((M,K))*0.06).astype(np.float32)
B=np.maximum(rng.standard_normal((K,N)),0).astype(np.float32)*np.float32(3.0)
B[:, :100] *= 1e-4
truth=A.astype(np.float64)@B.astype(np.float64)
norm=np.abs(A).astype(np.float64)@np.abs(B).astype(np.float64)
def rep(name,C):
    e=np.abs(C-truth)/norm; print(f"{name:10s} max {e.max():.2e} mean {e.mean():.2e}  rel|C| max {(np.abs(C-truth)/np.maximum(np.abs(truth),1e-30)).max():.2e}")
# fp32 sequential in blocks of 16 (mfma-like: exact block sum then fp32 add)
def acc_blocks(P):  # P: list of (Ai,Bi) pairs summed
    C=np.zeros((M,N),np.float32)
    for k0 in range(0,K,16):
        s=np.zeros((M,N),np.float64)
        for Ai,Bi in P: s+=Ai[:,k0:k0+16].astype(np.float64)@Bi[k0:k0+16].astype(np.float64)
        C=(C.astype(np.float64)+s).astype(np.float32)
    return C
rep("fp32mfma",acc_blocks([(A,B)]))
Ah=bf16(A);Al=bf16(A-Ah);Bh=bf16(B);Bl=bf16(B-Bh)
rep("bf16x3",acc_blocks([(Al,Bh),(Ah,Bl),(Ah,Bh)]))
Am=bf16(A-Ah-Al*0); Am=bf16(A-Ah); Al2=bf16(A-Ah-Am); Bm=bf16(B-Bh); Bl2=bf16(B-Bh-Bm)
rep("bf16x6",acc_blocks([(Al2,Bh),(Am,Bm),(Ah,Bl2),(Am,Bh),(Ah,Bm),(Ah,Bh)]))
# fp16x3 scaled: per-row A scale, per-col B scale to max in [2^14,2^15)
def sc(x,axis):
    m=np.abs(x).max(axis=axis,keepdims=True); e=np.floor(np.log2(np.maximum(m,1e-30))); return (2.0**(14-e)).astype(np.float32)
ra=sc(A,1); sb=sc(B,0)
As=A*ra; Bs=B*sb
Ah=f16(As);Al=f16(As-Ah);Bh=f16(Bs);Bl=f16(Bs-Bh)
C=acc_blocks([(Al,Bh),(Ah,Bl),(Ah,Bh)])
rep("fp16x3s",(C.astype(np.float64)/ra/sb).astype(np.float32))
