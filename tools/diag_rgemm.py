import os, sys
ROOT="/root/repo"
for p in (os.path.join(ROOT,"gguf-triton-kernel_amd"), os.path.join(ROOT,"oracle"), ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0,p)
import numpy as np, torch
import kernels._lib as kl
import oracle as O
from utils.synth import random_activations, random_blocks
dev=torch.device("cuda:0")
def prep(fmt,A,B,M,N,K):
    t=kl.TYPES[fmt]; ws=torch.empty(kl.workspace_size(t,M,N,K),dtype=torch.uint8,device=dev)
    kl.act_prepare(B,N,K,ws); C=kl.mmq_prepared(t,A,ws,M,N,K); torch.cuda.synchronize(); return C
for fmt in ("q8_0","q4_k","q6_k"):
  for N in (16,32,128):
    M,K=600,256
    qA=random_blocks(fmt,M,K,seed=N); B=random_activations(N,K,seed=N+1)
    A=torch.from_numpy(qA.view(np.int8)).to(dev); Bt=torch.from_numpy(B).to(dev)
    kl.set_tuning("GQ_RGEMM",1); C1=prep(fmt,A,Bt,M,N,K)
    kl.set_tuning("GQ_RGEMM",0); kl.set_tuning("GQ_WGEMM",0); kl.set_tuning("GQ_SKINNY",0); kl.set_tuning("GQ_GEMM_SPLITS",1)
    C0=prep(fmt,A,Bt,M,N,K); kl.reset_tuning()
    d=(C0.view(torch.int16)!=C1.view(torch.int16)).nonzero()
    ideal=O.mmq_from_fp16(fmt,qA,B,M,N,K,O.IDEAL)
    print(fmt,N,"mismatches",len(d),"rows",sorted(set(d[:,1].tolist()))[:20],"toks",sorted(set(d[:,0].tolist()))[:10],
          "err0",O.max_rel_err(C0.cpu().numpy(),ideal),"err1",O.max_rel_err(C1.cpu().numpy(),ideal), flush=True)
