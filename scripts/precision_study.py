"""CPU study: the head MLP with emulated split-bf16 products (as bf16 MFMAs would compute them)
through the PC sampler, against the reference's golden trajectories (tests/golden).

bf16x3 = (hi, mid) split, products hi*hi + hi*mid + mid*hi; bf16x6 = (hi, mid, lo) split, the six
products down to 2^-16 relative. Round-1 result (K=50/T=20 and K=10/T=100, rotation abs error):
fp32 1.9e-5 / 1.4e-6, bf16x3 4.3e-4 / 3.9e-5 (breaks the 1e-4 bar), bf16x6 1.35e-5 / 2.3e-6.
Usage: python scripts/precision_study.py
"""
import sys, numpy as np
import os
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0,ROOT); sys.path.insert(0,os.path.join(ROOT,'tests'))
from oracle import oracle
from genpose2_amd import weights
F32=np.float32
def bf16(a):
    a=np.ascontiguousarray(a,np.float32); b=a.view(np.uint32).astype(np.uint64)
    bias=0x7FFF+((b>>16)&1); r=((b+bias)&0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)
def split(a,n):
    out=[]; r=a.astype(F32)
    for _ in range(n):
        h=bf16(r); out.append(h); r=(r-h).astype(F32)
    return out
MODE=None
orig=oracle._lin
def lin_emul(x,w,b):
    if MODE is None: return orig(x,w,b)
    n, pairs = MODE
    xs=split(x,n); ws=split(w.astype(F32),n)
    acc=np.zeros((x.shape[0], w.shape[0]),np.float64)
    for i,j in pairs: acc += xs[i].astype(np.float64) @ ws[j].astype(np.float64).T
    return (acc.astype(F32) + b.astype(F32)).astype(F32)
oracle._lin=lin_emul
sd=weights.synthetic_state_dict("score")
import conftest
for name in ["pc_k50_t20","pc_k10_t100"]:
    g=conftest.golden(name); K,T=int(g["K"]),int(g["T"])
    for label,mode in [("fp32",None),("bf16x3",(2,[(0,0),(0,1),(1,0)])),("bf16x6",(3,[(0,0),(0,1),(1,0),(0,2),(1,1),(2,0)]))]:
        MODE=mode
        pose,q,feat,ex=oracle.pred_func(sd,g["pts"],g["pts_center"],K,T,"pc",g["prior"],g["z1"],g["z2"])
        ref=g["pred_pose"]
        rot=np.abs(pose[...,:6]-ref[...,:6]).max(); tr=np.abs(pose[...,6:]-ref[...,6:]).max()/np.abs(ref[...,6:]).max()
        print(name,label,"rot_abs",f"{rot:.2e}","trans_rel",f"{tr:.2e}",flush=True)
